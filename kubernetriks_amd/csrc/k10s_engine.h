// k10s_engine.h — one replica of kubernetriks' scheduling hot path + its event loop.
//
// Written once for the MI355X wavefront (64 lanes, wave-uniform control flow, lane-parallel node
// scans) and, with K10S_LANES == 1, for the host-side check build used only by tests.
//
// Reference semantics restated here (file:line of jellythefish/kubernetriks):
//   event queue        dslab-core (time, id) order, lazy cancel           SURVEY A.1
//   scheduling cycle   Scheduler::run_scheduling_cycle                     scheduler.rs:246-334
//   schedule_one       KubeScheduler::schedule_one + Fit + LeastAllocated  kube_scheduler.rs:68-151, plugin.rs:34-63
//   active queue       Rust BinaryHeap<QueuedPodInfo> sift order            queue.rs:29-33, SURVEY A.2
//   unschedulable map  BTreeMap<(ts total_cmp, name)>                       queue.rs:49-75
//   handlers           api_server.rs:127-457, persistent_storage.rs:185-490, scheduler.rs:382-477,
//                      node_component.rs:178-335, cluster_autoscaler.rs:230-334,
//                      kube_cluster_autoscaler.rs:62-326, horizontal_pod_autoscaler.rs:146-257,
//                      kube_horizontal_pod_autoscaler.rs:54-216, collector.rs:263-337,410-431
//   termination        RunUntilAllPodsAreFinishedCallbacks::on_step          simulation_callbacks.rs:86-91
#pragma once

#include "k10s_state.h"
#if !defined(__HIP__) && defined(K10S_PRUNE_STUDY)
#include <vector>
#endif

namespace k10s {

// ---- where a replica's inputs and working header live ------------------------------------------
// Device: the compiled scenario, the layout and the parameter/state base pointers of a launch sit
// in __constant__ memory (k10s_dc; scalar loads, no pointer chains through scratch), and the
// working replica header — clock, id counter, queue sizes, counters, estimators — is staged in LDS
// (k10s_hdr) for the whole launch: one workgroup = one replica.  Host (test-only check build): the
// same code reads them through the pointers held in Ctx.
// The replica region of this workgroup and its most used sections: by default (K10S_SEC_SGPR, Rep
// below) re-derived at each use from the workgroup id and the constant block (replica index x
// stride + section offset, SALU and scalar loads); with K10S_SEC_SGPR=0 read as absolute addresses
// from k10s_sec (LDS, written by the kernels before anything else) with one ds_read_b64 and two
// v_readfirstlane.
enum : int { SEC_BASE = 0, SEC_POD, SEC_NODE, SEC_SLOT, SEC_FQ, SEC_HEAP, SEC_SNODE, SEC_PRES, SEC_AQ, SEC_UQ,
             SEC_PARAMS, K10S_NSEC };   // SEC_PARAMS: this replica's k10s_replica_params (read-only)
#if defined(__HIP__)
__constant__ DevConst k10s_dc;
__shared__ RepHdr k10s_hdr;
__shared__ uint64_t k10s_sec[K10S_NSEC];
#endif

// ---- progress beacon (K10S_BEACON tooling builds) --------------------------------------------------
// Lane 0 of every replica writes the event it is about to handle (and the queue state) to host-mapped
// memory with system-scope stores before each dispatch, so a host thread can see where a launch that
// never returns stopped (tools/beacon_trace.py).  Product builds compile it out.
#ifndef K10S_BEACON
#define K10S_BEACON 0
#endif
#define K10S_BEACON_WORDS 16
#if defined(__HIP__) && K10S_BEACON
__device__ uint32_t* k10s_beacon;   // [replica][K10S_BEACON_WORDS], host-mapped (k10s_debug_beacon_alloc)
#endif

// ---- EXEC guard (K10S_EXEC_CHECK tooling builds) --------------------------------------------------
// Every lane-parallel helper (DPP/permlane reductions, ballots, readlane of a computed lane) assumes
// the whole wave is live: under a partial EXEC a DPP step reads the disabled partners' `old` value
// (0), so a reduction returns garbage, and a helper entered with an empty EXEC runs only its scalar
// control flow over stale vector values.  Check builds test EXEC at each such helper's entry (and
// bound the queue/heap sift loops: K10S_EXEC_CHECK bit 1); a violation stops the replica with K10S_ERR_EXEC_GUARD, site id
// in error_kind (| 0x100 when EXEC was empty).  The record is written with the whole wave switched on,
// because a vector store under an empty EXEC writes nothing.  Product builds compile it out.
#ifndef K10S_EXEC_CHECK
#define K10S_EXEC_CHECK 0
#endif
enum : uint32_t {
    XG_HEAP_POP = 1, XG_HEAP_MIN_CHILD, XG_HEAP_MIN_CHILD_EV, XG_SCHEDULE_SCAN, XG_SL_UPDATE, XG_FQ_REFILL,
    XG_PODS_IN_ORDER, XG_FOR_EACH_BIT, XG_CA_FIRST_FIT, XG_CA_SORT, XG_DISPATCH, XG_CYCLE, XG_GAUGE, XG_CACHE_FITS,
    XG_FAIR, XG_HANDLER, XG_EMIT, XG_SCAN_PLUGINS,
    XG_LOOP_HEAP_POP = 0x40, XG_LOOP_EMIT, XG_LOOP_AQ_POP, XG_LOOP_AQ_UP, XG_LOOP_STALE,
};
#if K10S_DEVICE && K10S_EXEC_CHECK
K10S_D bool exec_guard_fail(uint32_t site) {
#if defined(K10S_PLUGINS_TU)
    // (the plugins copy records with plain stores: the flat-address form below trips an instruction
    // selection error in that translation unit; an empty EXEC goes unrecorded there)
    k10s_hdr.error_code = K10S_ERR_EXEC_GUARD;
    k10s_hdr.error_kind = site;
    return false;
#else
    // generic (flat) addresses of the two header words: an LDS-aperture address works for flat stores
    const uint64_t a_code = (uint64_t)(uintptr_t)&k10s_hdr.error_code;
    const uint64_t a_kind = (uint64_t)(uintptr_t)&k10s_hdr.error_kind;
    const uint32_t code = K10S_ERR_EXEC_GUARD;
    uint64_t saved, va;
    uint32_t vd;
    asm volatile(
        "s_or_saveexec_b64 %0, -1\n\t"
        "v_mov_b32 %1, %3\n\t"
        "v_mov_b64 %2, %4\n\t"
        "flat_store_dword %2, %1\n\t"
        "v_mov_b32 %1, %5\n\t"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
        "v_mov_b64 %2, %6\n\t"
        "flat_store_dword %2, %1\n\t"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved), "=&v"(vd), "=&v"(va)
        : "s"(code), "s"(a_code), "s"(site), "s"(a_kind)
        : "memory");
    return false;
#endif
}
// true when the whole wave is live; otherwise records the site and returns false (the caller returns)
K10S_D bool exec_guard(uint32_t site) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if (__builtin_expect(ex == ~0ull, 1)) return true;
    return exec_guard_fail(site | (ex == 0 ? 0x100u : 0u));
}
// K10S_EXEC_CHECK bit 0: the entry guards; bit 1: the loop bounds (each alone perturbs codegen less)
#if K10S_EXEC_CHECK & 1
#define K10S_FULL_WAVE(site) exec_guard(site)
#else
#define K10S_FULL_WAVE(site) true
#endif
#if K10S_EXEC_CHECK & 2
// a bounded loop took more than `cap` iterations (it = the loop's counter)
#define K10S_LOOP_CAP(it, cap, site) (++(it) > (cap) ? exec_guard_fail(site), true : false)
#else
#define K10S_LOOP_CAP(it, cap, site) false
#endif
#else
#define K10S_FULL_WAVE(site) true
#define K10S_LOOP_CAP(it, cap, site) false
#endif
// Every read of the launch constants goes through an opaque copy of the block's address (an empty
// asm the compiler cannot see through): the scalar loads are then issued where a value is used
// instead of being hoisted out of the event loop and kept live across it, which is what
// exhausted the SGPRs (and spilled them into VGPR lanes) and raised the loop's VGPR count.
#if K10S_DEVICE
typedef const __attribute__((address_space(4))) DevConst* DevConstPtr;
K10S_D DevConstPtr dc_ptr() {
    DevConstPtr p = (DevConstPtr)&k10s_dc;
    asm volatile("" : "+s"(p));
    return p;
}
#define K10S_DC (*dc_ptr())
#endif

// Typed accessors over one replica's region; section bases are recomputed from the (constant)
// layout at each use instead of being held live across the event loop.
// K10S_SEC_SGPR=1 (default since round 5): a section base is the workgroup id (one replica per
// workgroup) x the stride + the section's offset, from the constant block: scalar loads and SALU
// only, where the LDS table costs a ds_read_b64 and two v_readfirstlane per use.  The handlers'
// VALU falls 10-20 % statically for 20-30 % more SALU (C3 +0.9 %, backlog +1.8 %,
// profiles/r05_ab13_sec_sgpr.json).  0: the LDS table k10s_sec.
#ifndef K10S_SEC_SGPR
#define K10S_SEC_SGPR 1
#endif
struct Rep {
#if K10S_DEVICE
#if K10S_SEC_SGPR
    K10S_D static K10S_GB(uint8_t) sec(int i) {
        const DevConst& D = K10S_DC;
        // a callee receives the id in an SGPR, the kernel keeps it across its calls; the empty asm
        // makes every use recompute the base instead of hoisting r x stride out of the event loop
        // and keeping it live (in VGPRs) across the handler calls
        uint32_t r = (uint32_t)__builtin_amdgcn_readfirstlane((int)__builtin_amdgcn_workgroup_id_x());
        asm volatile("" : "+s"(r));
        if (i == SEC_PARAMS) return (K10S_GB(uint8_t))(D.params + r);
        const Layout& L = D.L;
        const uint64_t off = i == SEC_POD ? L.pod : i == SEC_NODE ? L.node : i == SEC_SLOT ? L.slot : i == SEC_FQ ? L.fq
                           : i == SEC_HEAP ? L.heap : i == SEC_SNODE ? L.s_node : i == SEC_PRES ? L.s_present
                           : i == SEC_AQ ? L.aq : i == SEC_UQ ? L.uq : 0;
        return (K10S_GB(uint8_t))((uint64_t)D.base + (uint64_t)r * L.stride + off);
    }
#else
    K10S_D static K10S_GB(uint8_t) sec(int i) { return (K10S_GB(uint8_t))uniform_u64(k10s_sec[i]); }
#endif
    K10S_D const Layout& L() const { return K10S_DC.L; }
    template <typename T>
    K10S_D T* at(uint64_t off) const { return (T*)(sec(SEC_BASE) + off); }
    // a section with its own entry in k10s_sec (the offset argument is the host's)
    template <typename T>
    K10S_D T* hot(int i, uint64_t) const { return (T*)sec(i); }
#else
    uint8_t* b;
    const Layout* Lp;
    const Layout& L() const { return *Lp; }
    template <typename T>
    T* at(uint64_t off) const { return (T*)(b + off); }
    template <typename T>
    T* hot(int, uint64_t off) const { return at<T>(off); }
#endif
    K10S_HD RepHdr* h() const { return at<RepHdr>(L().hdr); }
    K10S_HD uint64_t* s_node() const { return hot<uint64_t>(SEC_SNODE, L().s_node); }
    K10S_HD uint64_t* fr_val() const { return at<uint64_t>(L().fr_val); }
    K10S_HD uint8_t* fr_idx() const { return at<uint8_t>(L().fr_idx); }
    K10S_HD uint32_t* s_cpu() const { return at<uint32_t>(L().s_cpu); }
    K10S_HD uint64_t* s_ram() const { return at<uint64_t>(L().s_ram); }
    K10S_HD uint64_t* s_present() const { return hot<uint64_t>(SEC_PRES, L().s_present); }
    K10S_HD uint32_t* s_bcpu() const { return at<uint32_t>(L().s_bcpu); }
    K10S_HD uint32_t* s_ccpu() const { return at<uint32_t>(L().s_ccpu); }
    K10S_HD uint64_t* s_cram() const { return at<uint64_t>(L().s_cram); }
    K10S_HD uint64_t* s_bram() const { return at<uint64_t>(L().s_bram); }
    K10S_HD NodeState& node(uint32_t n) const { return hot<NodeState>(SEC_NODE, L().node)[n]; }
    K10S_HD uint64_t* pend_rm() const { return at<uint64_t>(L().pend_rm); }
    K10S_HD PodState& pod(uint32_t p) const { return hot<PodState>(SEC_POD, L().pod)[p]; }
    K10S_HD k10s_pod_record* prec() const { return L().rec_on ? at<k10s_pod_record>(L().prec) : nullptr; }
    K10S_HD SlotState& slot(int32_t s) const { return hot<SlotState>(SEC_SLOT, L().slot)[s]; }
    K10S_HD uint32_t* pool_ring() const { return at<uint32_t>(L().pool_ring); }
    K10S_HD GroupState* grp() const { return at<GroupState>(L().grp); }
    K10S_HD uint64_t* grp_bits() const { return at<uint64_t>(L().grp_bits); }
    K10S_HD uint32_t* cag() const { return at<uint32_t>(L().cag); }
    K10S_HD CAAct* ca_act() const { return at<CAAct>(L().ca_act); }
    K10S_HD uint32_t* ca_cpu() const { return at<uint32_t>(L().ca_cpu); }
    K10S_HD uint64_t* ca_ram() const { return at<uint64_t>(L().ca_ram); }
    K10S_HD uint32_t* ca_undo() const { return at<uint32_t>(L().ca_undo); }
    K10S_HD uint64_t* ca_ubits() const { return at<uint64_t>(L().ca_ubits); }
    K10S_HD uint64_t* ca_live() const { return at<uint64_t>(L().ca_live); }
    K10S_HD int32_t* ps_head() const { return at<int32_t>(L().ps_head); }
    K10S_HD int32_t* ps_link() const { return at<int32_t>(L().ps_link); }   // [2p] prev, [2p + 1] next
    K10S_HD uint32_t* ca_list() const { return at<uint32_t>(L().ca_list); }
    K10S_HD HeapEv* heap() const { return hot<HeapEv>(SEC_HEAP, L().heap); }
    K10S_HD HeapEv* fq() const { return hot<HeapEv>(SEC_FQ, L().fq); }
    K10S_HD QInfo* aq() const { return hot<QInfo>(SEC_AQ, L().aq); }
    K10S_HD QInfo* uq() const { return hot<QInfo>(SEC_UQ, L().uq); }
    K10S_HD k10s_log_entry* log() const { return L().cap_log ? at<k10s_log_entry>(L().log) : nullptr; }
    K10S_HD k10s_placement* place() const { return L().cap_place ? at<k10s_placement>(L().place) : nullptr; }
    K10S_HD k10s_gauge_row* gauge() const { return at<k10s_gauge_row>(L().gauge); }
    K10S_HD uint32_t* g_cpu() const { return at<uint32_t>(L().g_cpu); }
    K10S_HD uint64_t* g_ram() const { return at<uint64_t>(L().g_ram); }
};

#if !K10S_DEVICE
inline Rep make_rep(uint8_t* base, const Layout& L, uint32_t r) {
    Rep v;
    v.b = base + (uint64_t)r * L.stride;
    v.Lp = &L;
    return v;
}
#endif

// The handlers' view of the current replica.  Mutable simulation registers (clock, next id, queue
// sizes, trace cursor, sticky error) are fields of the working header H().
struct Ctx {
#if K10S_DEVICE
    K10S_D const Scenario& S() const { return K10S_DC.sc; }
    K10S_D const Params& P() const { return *(K10S_RO(Params))Rep::sec(SEC_PARAMS); }
    K10S_D const Layout& Ly() const { return K10S_DC.L; }
    K10S_D RepHdr& H() const { return k10s_hdr; }
    K10S_D Rep V() const { return Rep(); }
#else
    const Scenario* sc;
    const Params* pr;
    RepHdr* h;
    Rep v;
    const Layout* Lp;
    const Scenario& S() const { return *sc; }
    const Params& P() const { return *pr; }
    const Layout& Ly() const { return *Lp; }
    RepHdr& H() const { return *h; }
    Rep V() const { return v; }
#endif
};

K10S_HD void fail(Ctx& c, uint32_t code) {
#if K10S_DEVICE
    // the code is materialized here, on the (cold) error path: as a plain constant the compiler
    // hoisted each code's VGPR copy out of the event loop and held six of the loop's 64 VGPRs with them
    asm volatile("" : "+s"(code));
#endif
    RepHdr& h = c.H();
    if (h.error_code == 0) {
        h.error_code = code;
        h.error_kind = h.cur_kind;
        h.error_seq = h.cur_seq;
        h.error_time = h.clock;
    }
}

// Runs of one event kind handled together (defined with the event queue below); called by the
// handlers of the run kinds.
// (tuning knob, semantics-neutral: 0 = every event one by one)
#ifndef K10S_RUNS
#define K10S_RUNS 1
#endif
K10S_HD_NOINL uint32_t run_batch(Ctx& c, uint32_t k);
K10S_HD_NOINL uint32_t win_batch(Ctx& c);
#define K10S_RUN_CALL(c, k) (uniform_u32(run_batch((c), (k))) != 0u)

// ---- the scheduler's node cache (allocatable per node in name order: the scan target) -----------
// Two layouts of the same values (Layout.packed, chosen per engine by make_layout):
//  * packed: one u64 per node, cpu in bits 40..63, ram in bits 0..39 (every node definition of the
//    scenario has cpu < 2^24 and ram < 2^40, and allocatable <= capacity), so a scan streams 8 B
//    per node instead of 12 and a reservation is one 64-bit subtraction;
//  * wide: the u32 cpu + u64 ram SoA (larger nodes, pruned scans, and the score-plugin kernel, which
//    also reads the capacity SoA).
// Device: k10s_kernels.hip is compiled packed-only and k10s_kernels_plugins.hip wide-only
// (K10S_PACKED); the host check build follows the layout at run time.
#define K10S_PK_SHIFT 40
#define K10S_PK_RAM ((1ull << K10S_PK_SHIFT) - 1)
#define K10S_PK_CPU ((1u << (64 - K10S_PK_SHIFT)) - 1)
#if K10S_DEVICE
#ifndef K10S_PACKED
#define K10S_PACKED 1
#endif
K10S_HD constexpr bool nc_packed(const Ctx&) { return K10S_PACKED != 0; }
#else
inline bool nc_packed(const Ctx& c) { return c.Ly().packed != 0; }
#endif
struct NcEnt {
    uint32_t cpu;
    uint64_t ram;
};
K10S_HD uint64_t nc_pack(uint32_t cpu, uint64_t ram) { return ((uint64_t)cpu << K10S_PK_SHIFT) | ram; }
K10S_HD NcEnt nc_unpack(uint64_t x) {
    NcEnt v;
    v.cpu = (uint32_t)(x >> K10S_PK_SHIFT);
    v.ram = x & K10S_PK_RAM;
    return v;
}
K10S_HD NcEnt nc_get(Ctx& c, uint32_t n) {
    if (nc_packed(c)) return nc_unpack(c.V().s_node()[n]);
    NcEnt v;
    v.cpu = c.V().s_cpu()[n];
    v.ram = c.V().s_ram()[n];
    return v;
}
// (cpu, ram) must fit the packed fields when packed (every caller stores allocatable <= capacity,
// or 0, or checks with nc_release)
K10S_HD void nc_put(Ctx& c, uint32_t n, NcEnt v) {
    if (nc_packed(c)) {
        c.V().s_node()[n] = nc_pack(v.cpu, v.ram);
    } else {
        c.V().s_cpu()[n] = v.cpu;
        c.V().s_ram()[n] = v.ram;
    }
}
// A packed entry of node n changed: its 64-node block's front is stale (front_scan).  Wave-uniform
// callers only (a lane-parallel writer ORs its blocks into fr_dirty itself: run_batch).
#ifndef K10S_FRONT
#define K10S_FRONT 1   // A/B knob: 0 = every fast-path attempt scans the whole cache (round 5)
#endif
K10S_HD void fr_mark(Ctx& c, uint32_t n) {
    if (K10S_FRONT && c.Ly().front) c.H().fr_dirty |= 1ull << (n >> 6);
}
// reserve_node_resources (scheduler.rs:118-123) after Fit: request <= allocatable, no borrow
K10S_HD void nc_reserve(Ctx& c, uint32_t n, uint32_t rc, uint64_t rr) {
    if (nc_packed(c)) {
        fr_mark(c, n);
        c.V().s_node()[n] -= nc_pack(rc, rr);
    } else {
        c.V().s_cpu()[n] -= rc;
        c.V().s_ram()[n] -= rr;
    }
}
// release_node_resources (scheduler.rs:153-162) onto entry v of node n: false (and the replica
// stops with K10S_ERR_NODE_CACHE_RANGE) if a packed field would overflow
K10S_HD bool nc_release(Ctx& c, uint32_t n, NcEnt v, uint32_t rc, uint64_t rr) {
    if (nc_packed(c)) {
        if (rc > K10S_PK_CPU - v.cpu || rr > K10S_PK_RAM - v.ram) {
            fail(c, K10S_ERR_NODE_CACHE_RANGE);
            return false;
        }
        fr_mark(c, n);
        c.V().s_node()[n] = nc_pack(v.cpu + rc, v.ram + rr);
    } else {
        c.V().s_cpu()[n] = v.cpu + rc;
        c.V().s_ram()[n] = v.ram + rr;
    }
    return true;
}

// Broadcast an event loaded by vector loads to scalar registers: every field is wave-uniform by
// construction, and saying so lets every address derived from it be computed on the scalar unit.
K10S_HD void uniform_event(HeapEv& e) {
#if K10S_DEVICE
    uint64_t tb = f2u(e.time);
    e.time = u2f(((uint64_t)uniform_u32((uint32_t)(tb >> 32)) << 32) | uniform_u32((uint32_t)tb));
    e.seq = uniform_u32(e.seq);
    uint32_t ks = uniform_u32((uint32_t)e.kind | ((uint32_t)(uint16_t)e.slot << 16));
    e.kind = (uint16_t)ks;
    e.slot = (int16_t)(ks >> 16);
    e.a = uniform_u32(e.a);
    e.b = uniform_u32(e.b);
    uint64_t xb = f2u(e.x);
    e.x = u2f(((uint64_t)uniform_u32((uint32_t)(xb >> 32)) << 32) | uniform_u32((uint32_t)xb));
#else
    (void)e;
#endif
}

// How an event reaches its out-of-line handler: as the address of its LDS copy (the head entry of
// its source, which the loop consumes only after the handler ran; a trace event is first written to
// the header's cur_ev slot), so a call passes one 32-bit VGPR and the loop reads only the fields it
// tests (round 2 passed the event by value in 8 VGPRs, each handler reading them to SGPRs again).
#if K10S_DEVICE
typedef const __attribute__((address_space(3))) HeapEv* EvRef;
#define K10S_EVREF(x) ((EvRef)(x))
#else
typedef const HeapEv* EvRef;
#define K10S_EVREF(x) ((EvRef)(x))
#endif
#define K10S_EVARG EvRef ep
// Device: a handler reads each field of its event where a case uses it (an LDS read and its
// readfirstlanes at the use) instead of all eight fields up front: C3 1,215 -> 1,203 ms
// (profiles/r04_t1_ab.json).
#if K10S_DEVICE
struct EvLazy {
    EvRef ep;
    struct U32 {
        const __attribute__((address_space(3))) uint32_t* p;
        K10S_D operator uint32_t() const { return uniform_u32(*p); }
    };
    struct F64 {
        const __attribute__((address_space(3))) double* p;
        K10S_D operator double() const { return uniform_f64(*p); }
    };
    struct Kind {
        const __attribute__((address_space(3))) uint32_t* p;
        K10S_D operator uint32_t() const { return uniform_u32(*p) & 0xFFFFu; }
    };
    struct Slot {
        const __attribute__((address_space(3))) uint32_t* p;
        K10S_D operator int32_t() const { return (int32_t)(int16_t)(uniform_u32(*p) >> 16); }
    };
    F64 time;
    U32 seq;
    Kind kind;
    Slot slot;
    U32 a, b;
    F64 x;
    K10S_D explicit EvLazy(EvRef e)
        : ep(e), time{&e->time}, seq{&e->seq}, kind{(const __attribute__((address_space(3))) uint32_t*)&e->kind},
          slot{(const __attribute__((address_space(3))) uint32_t*)&e->kind}, a{&e->a}, b{&e->b}, x{&e->x} {}
};
#define K10S_EV_PROLOGUE                     \
    if (!K10S_FULL_WAVE(XG_HANDLER)) return; \
    const EvLazy e(ep)
#else
#define K10S_EV_PROLOGUE                     \
    if (!K10S_FULL_WAVE(XG_HANDLER)) return; \
    HeapEv e = *ep;                          \
    uniform_event(e)
#endif

// ---- cycle attribution (K10S_PROF builds: tooling only, semantics-neutral) ----------------------
// s_memtime deltas per loop phase, accumulated in RepHdr::prof and read by k10s_engine_profile.
enum : int { PROF_LOOP = 0, PROF_SELECT = 1, PROF_CONSUME = 2, PROF_DISPATCH = 3, PROF_CYCLE = 4, PROF_SCAN = 5,
             PROF_NSCAN = 6, PROF_BOUNDS = 7, PROF_AQPOP = 8, PROF_HEAPPOP = 9, PROF_NHEAPPOP = 10, PROF_EMIT = 11,
             PROF_NEMIT = 12, PROF_AQPUSH = 13, PROF_WFRONT = 14, PROF_WAPPLY = 15 };
K10S_HD uint64_t prof_now() {
#if K10S_PROF && K10S_DEVICE
    // an ordered read (volatile, memory clobber): the builtin's reads could move across the code they
    // bracket once that code was inlined (round 4's c5_autoscaled profile had a corrupt phase slot)
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    return t;
#else
    return 0;
#endif
}
#if K10S_PROF
#define K10S_PROF_ADD(c, slot, t0) ((c).H().prof[(slot)] += prof_now() - (t0))
#define K10S_PROF_COUNT(c, slot) ((c).H().prof[(slot)] += 1)
#else
#define K10S_PROF_ADD(c, slot, t0) ((void)(t0))
#define K10S_PROF_COUNT(c, slot) ((void)0)
#endif

// ---- small helpers ---------------------------------------------------------------------------
K10S_HD bool bit_test(const uint64_t* w, uint32_t i) { return (w[i >> 6] >> (i & 63)) & 1ull; }
K10S_HD void bit_set(uint64_t* w, uint32_t i) { w[i >> 6] |= (1ull << (i & 63)); }
K10S_HD void bit_clear(uint64_t* w, uint32_t i) { w[i >> 6] &= ~(1ull << (i & 63)); }

K10S_HD bool is_multiple_of_1000(double x) {
    // fmod(x, 1000.0) == 0.0 for a simulation clock (finite, >= 0, < 2^63)
    if (!(x >= 0.0) || x >= 9.2e18) return false;
    double fl = __builtin_floor(x);
    if (fl != x) return false;
    return ((uint64_t)x % 1000ull) == 0;
}

K10S_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ---- dslab event queue: binary min-heap on (time total order, id) ------------------------------
K10S_HD bool ev_before(double ta, uint32_t sa, double tb, uint32_t sb) {
    int64_t ka = total_key(ta), kb = total_key(tb);
    return ka < kb || (ka == kb && sa < sb);
}

// The dslab queue as a K10S_HEAP_D-ary (default 64) min-heap of 32-B events.  Ids are unique, so
// every arity pops the same (time, id) order; a wide heap cuts the dependent load chain of a pop to
// ~log_D(n) levels, and the D children of a level (contiguous) are loaded and compared by D lanes
// at once.

// Delay classes: every emission site with a constant network delay (or delay 0) names its class;
// emissions of one class happen in nondecreasing clock order, so clock + delay is nondecreasing
// and ids increase: each class is a sorted run and goes to its FIFO ring.  An entry that would
// break the run (a variable delay, or a full ring) goes to the heap instead, so correctness never
// depends on the classification.  Ticks, the scheduling cycle and pod-finish self-events (variable
// delays) always use the heap.
enum : int {
    FQ_HEAP = -1,
    FQ_AS_TO_PS = 0,     // api server <-> persistent storage
    FQ_PS_TO_SCHED = 1,  // persistent storage -> scheduler
    FQ_SCHED_TO_AS = 2,  // scheduler -> api server (PodNotScheduled)
    FQ_ASSIGN = 3,       // scheduler -> api server (AssignPodToNodeRequest: cycle offset + delay)
    FQ_AS_TO_NODE = 4,   // api server <-> node components
    FQ_AS_TO_CA = 5,     // cluster autoscaler / HPA actions
    FQ_AS_TO_HPA = 6,
    FQ_NOW = 7,          // emit_now (delay 0)
};
// The other two event sources: the shared trace stream and the heap.
enum : int { SRC_TRACE = K10S_NFQ, SRC_HEAP = K10S_NFQ + 1 };

// Heap position i: the top K10S_HEAP_TOP positions (levels 0-1; 0-2 for arity 8) are in the working
// header, the rest in the replica's HBM heap array.  Level boundaries coincide with K10S_HEAP_TOP,
// so the children of one node are either all in the header or all in HBM.
static_assert(K10S_HEAP_D != 8 || K10S_HEAP_TOP == 1 + K10S_HEAP_D + K10S_HEAP_D * K10S_HEAP_D, "heap top = levels 0..2");
static_assert(K10S_HEAP_D == 8 || K10S_HEAP_TOP == 1 + K10S_HEAP_D, "heap top = levels 0..1");
// Device: both arrays are reached through address-space-typed pointers (LDS symbol, global
// pointer), so the compiler can never merge the two paths into one generic (FLAT) access.
#if K10S_DEVICE
// HBM part through a raw buffer descriptor (scalar base, 32-bit offsets): distinct instructions
// from the LDS path, so the two are never merged into one generic (FLAT) access.
K10S_D __amdgpu_buffer_rsrc_t heap_rsrc(Ctx& c) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)c.V().heap(), (short)0,
                                             (int)(K10S_DC.L.cap_heap * (uint32_t)sizeof(HeapEv)), 0x00020000);
}
// The HBM part is a structure of two arrays (round 5): position i's key half (time, id, kind|slot;
// 16 B) at i·16 and its payload half (a, b, x; 16 B) at (cap_heap + i)·16, both in the heap section
// (cap_heap · 32 B, as sized by the builder).  A pop's minimum over 64 children then reads only key
// halves — 1 KB a level instead of 2 KB — and the chosen child's payload (heap_min_child_ev).
// Device-only: the host engine's heap stays an array of HeapEv (no state crosses the two).
static_assert(sizeof(HeapEv) == 32, "key and payload halves of 16 B");
K10S_D int heap_key_off(uint32_t i) { return (int)(i * 16u); }
K10S_D int heap_pay_off(uint32_t i) { return (int)((K10S_DC.L.cap_heap + i) * 16u); }
K10S_D HeapEv heap_get(Ctx& c, uint32_t i) {
    if (i < K10S_HEAP_TOP) return k10s_hdr.heap_lds[i];
    const __amdgpu_buffer_rsrc_t rs = heap_rsrc(c);
    auto lo = __builtin_amdgcn_raw_buffer_load_b128(rs, heap_key_off(i), 0, 0);
    auto hi = __builtin_amdgcn_raw_buffer_load_b128(rs, heap_pay_off(i), 0, 0);
    HeapEv e;
    e.time = u2f(((uint64_t)lo[1] << 32) | lo[0]);
    e.seq = lo[2];
    e.kind = (uint16_t)lo[3];
    e.slot = (int16_t)(lo[3] >> 16);
    e.a = hi[0];
    e.b = hi[1];
    e.x = u2f(((uint64_t)hi[3] << 32) | hi[2]);
    return e;
}
K10S_D void heap_put(Ctx& c, uint32_t i, const HeapEv& e) {
    if (i < K10S_HEAP_TOP) {
        k10s_hdr.heap_lds[i] = e;
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = heap_rsrc(c);
    const uint64_t tb = f2u(e.time), xb = f2u(e.x);
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    v4u lo = {(uint32_t)tb, (uint32_t)(tb >> 32), e.seq, (uint32_t)e.kind | ((uint32_t)(uint16_t)e.slot << 16)};
    v4u hi = {e.a, e.b, (uint32_t)xb, (uint32_t)(xb >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(lo, rs, heap_key_off(i), 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rs, heap_pay_off(i), 0, 0);
}
#else
K10S_HD HeapEv heap_get(Ctx& c, uint32_t i) { return i < K10S_HEAP_TOP ? c.H().heap_lds[i] : c.V().heap()[i]; }
K10S_HD void heap_put(Ctx& c, uint32_t i, const HeapEv& e) {
    if (i < K10S_HEAP_TOP) c.H().heap_lds[i] = e;
    else c.V().heap()[i] = e;
}
#endif

// Host-only event statistics (tooling: tools/host_stats.py builds the host engine with
// -DK10S_HOST_STATS and reads k10s_host_stats); compiled out everywhere else.
#if !K10S_DEVICE && defined(K10S_HOST_STATS)
extern "C" uint64_t k10s_host_stats[48];
#define K10S_HSTAT(i) (k10s_host_stats[i] += 1)
#else
#define K10S_HSTAT(i) ((void)0)
#endif
// Host-only memory-touch model (tooling: tools/traffic_model.py builds the host engine with
// -DK10S_TRAFFIC_MODEL and compiler load/store tracing; the runtime attributes every touched line of
// the replica's HBM sections to the kind of the event the loop is handling); compiled out elsewhere.
#if !K10S_DEVICE && defined(K10S_TRAFFIC_MODEL)
extern "C" void k10s_tm_replica(const void* base, const void* layout);
extern "C" void k10s_tm_event(uint32_t kind);
#define K10S_TM_EVENT(k) k10s_tm_event(k)
#else
#define K10S_TM_EVENT(k) ((void)0)
#endif
enum { HS_EVENTS, HS_FIFO_POP, HS_REFILL, HS_HEAP_POP, HS_TRACE_POP, HS_SL_FAST, HS_SL_UPDATE, HS_EMIT_WIN,
       HS_EMIT_RING, HS_EMIT_HEAP, HS_SL_DIRTY, HS_SCANS, HS_REFILL_CLS0 = 12, HS_POP_CLS0 = 20, HS_AQ_HBM_GET = 28, HS_AQ_POP = 29, HS_SLPOS0 = 32,
       HS_NEXT_EMITTED = 36, HS_NEXT_EMITTED_FIFO = 37, HS_RUNS = 38, HS_RUN_EVENTS = 39, HS_RUN_REFUSED = 40,
       HS_WINDOWS = 41, HS_WIN_EVENTS = 42, HS_TILE_PICKS = 43, HS_TILE_RESCANS = 44, HS_FUSED_FINISH = 45 };
// An emission changed source q's head: mark it for the source list.
K10S_HD void sl_mark(RepHdr& H, uint32_t q) { H.sl_dirty |= 1u << q; }
K10S_HD void pods_left_dec(RepHdr& H) { H.pods_left -= 1; }

K10S_HELPER uint32_t emit(Ctx& c, uint32_t kind, double delay, int32_t slot, uint32_t a, uint32_t b, double x,
                          int cls = FQ_HEAP) {
    RepHdr& H = c.H();
    // Everything emit reads from the header and the launch constants, as one batch ahead of every
    // branch (the compiler may not hoist loads above the early returns): one LDS/scalar round trip
    // instead of one per field.
    const uint32_t err = H.error_code, seq = H.next_seq, hsize = H.heap_size;
    const double clock = H.clock;
    const uint32_t cap = c.Ly().cap_fq, cap_heap = c.Ly().cap_heap;
    uint32_t hd = 0, tl = 0, we = 0;
    double last = 0.0;
    if (cls >= 0) {
        hd = H.fq[cls].head;
        tl = H.fq[cls].tail;
        we = H.fq[cls].wend;
        last = H.fq[cls].last;
    }
    if (err) return 0;
    if (seq == 0xFFFFFFFFu) {
        fail(c, K10S_ERR_SEQ_OVERFLOW);
        return 0;
    }
#if !K10S_TIME_KEY_ID
    // dslab-core add_event refuses an event in the past (a negative or NaN delay) with a panic.  Only
    // the signed-time copies check: the default kernel copy runs scenarios whose every delay, interval,
    // duration and trace time is >= 0 (times_nonneg, k10s_builder.cpp), where no emission can be.
    // (This also keeps the events-by-reference rule: an emission never precedes the event handled.)
    if (!(delay >= 0.0)) {
        fail(c, K10S_PANIC_NEGATIVE_DELAY);
        return 0;
    }
#endif
    HeapEv e;
    e.time = clock + delay;
    e.seq = seq;
    e.kind = (uint16_t)kind;
    e.slot = (int16_t)slot;
    e.a = a;
    e.b = b;
    e.x = x;
    const int64_t k = total_key(e.time);
    if (cls >= 0 && cap) {
        if (tl - hd < cap && (tl == hd || k >= total_key(last))) {
            if (we == tl && tl - hd < K10S_FQW) {  // the window holds the whole ring: append
                H.fq_win[(uint32_t)cls * K10S_FQW + (tl & (K10S_FQW - 1))] = e;
                H.fq[cls].wend = tl + 1;
                K10S_HSTAT(HS_EMIT_WIN);
            } else {
                c.V().fq()[(uint32_t)cls * cap + (tl & (cap - 1))] = e;
                K10S_HSTAT(HS_EMIT_RING);
            }
            if (tl == hd) sl_mark(H, (uint32_t)cls);  // the ring was empty: a new head (source list)
            H.fq[cls].tail = tl + 1;
            H.fq[cls].last = e.time;
            H.next_seq = e.seq + 1;
            return e.seq;
        }
    }
    if (hsize >= cap_heap) {
        fail(c, K10S_ERR_HEAP_FULL);
        return 0;
    }
    H.next_seq = e.seq + 1;
    K10S_HSTAT(HS_EMIT_HEAP);
    uint32_t pos = uniform_u32(hsize);
    H.heap_size = pos + 1;
    [[maybe_unused]] uint32_t it = 0;
    while (pos > 0) {
        if (K10S_LOOP_CAP(it, 12, XG_LOOP_EMIT)) break;
        uint32_t parent = (pos - 1) / K10S_HEAP_D;
        HeapEv p = heap_get(c, parent);
        uniform_event(p);  // wave-uniform by construction: keep the sift loop on the scalar unit
        int64_t kp = total_key(p.time);
        if (!(k < kp || (k == kp && e.seq < p.seq))) break;
        heap_put(c, pos, p);
        pos = parent;
    }
    heap_put(c, pos, e);
    if (pos == 0) {  // a new heap root (source list update)
        H.heap_top = e;
        sl_mark(H, SRC_HEAP);
    }
    return e.seq;
}
K10S_HD uint32_t emit0(Ctx& c, uint32_t kind, double delay) { return emit(c, kind, delay, -1, 0, 0, 0.0); }

// Smallest (time, id) among children [first, min(first + D, n)); returns its index.  Device: lanes
// 0..D-1 load one child's key each (one contiguous read) and reduce with log2(D) DPP/permlane steps.
K10S_HD uint32_t heap_min_child(Ctx& c, uint32_t first, uint32_t n, int64_t& kmin, uint32_t& smin) {
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_HEAP_MIN_CHILD)) {
        kmin = 0x7FFFFFFFFFFFFFFFll;
        smin = 0xFFFFFFFFu;
        return first;
    }
    const int lane = lane_id();
    uint32_t i = first + (uint32_t)(lane & (K10S_HEAP_D - 1));
    int64_t k = 0x7FFFFFFFFFFFFFFFll;
    uint32_t sq = 0xFFFFFFFFu;
    if (lane < K10S_HEAP_D && i < n) {
        if (first < K10S_HEAP_TOP) {
            k = total_key(k10s_hdr.heap_lds[i].time);
            sq = k10s_hdr.heap_lds[i].seq;
        } else {
            const __amdgpu_buffer_rsrc_t rs = heap_rsrc(c);
            auto lo = __builtin_amdgcn_raw_buffer_load_b128(rs, heap_key_off(i), 0, 0);
            k = total_key(u2f(((uint64_t)lo[1] << 32) | lo[0]));
            sq = lo[2];
        }
    }
    keymin_step<0>(k, sq, i);
    keymin_step<1>(k, sq, i);
    keymin_step<2>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 16) keymin_step<3>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 32) keymin_step<4>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 64) keymin_step<5>(k, sq, i);
    // lanes 0..D-1 now agree; broadcast lane 0's result to the whole wave
    const uint64_t klo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)k);
    const uint64_t khi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)k >> 32));
    kmin = (int64_t)(klo | (khi << 32));
    smin = (uint32_t)__builtin_amdgcn_readfirstlane((int)sq);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
#else
    uint32_t best = first;
    HeapEv f = heap_get(c, first);
    int64_t kb = total_key(f.time);
    uint32_t sb = f.seq;
    uint32_t end = first + K10S_HEAP_D < n ? first + K10S_HEAP_D : n;
    for (uint32_t i = first + 1; i < end; i++) {
        HeapEv h = heap_get(c, i);
        int64_t k = total_key(h.time);
        if (k < kb || (k == kb && h.seq < sb)) {
            kb = k;
            sb = h.seq;
            best = i;
        }
    }
    kmin = kb;
    smin = sb;
    return best;
#endif
}

#if K10S_DEVICE
// The device's heap_pop: (a) the moved-up entry of a level in HBM: its key half taken from the
// lane that loaded it (heap_min_child_ev loads the 64 children's key halves) and its payload half
// loaded once the minimum is known, and (b) the last entry's load awaited only after the first
// level's minimum (LDS) is known.
// Same comparisons and moves.  Inlined into the event loop it lost 1.5 % to register pressure
// (profiles/r03_k6_heap_pop_ab.json); the whole pop runs out of line on the device (+1.6 %,
// profiles/r03_k11_heap_pop_call_ab.json).
K10S_D uint32_t heap_min_child_ev(Ctx& c, uint32_t first, uint32_t n, int64_t& kmin, uint32_t& smin, HeapEv& ev) {
    if (!K10S_FULL_WAVE(XG_HEAP_MIN_CHILD_EV)) {
        kmin = 0x7FFFFFFFFFFFFFFFll;
        smin = 0xFFFFFFFFu;
        return first;
    }
    if (first < K10S_HEAP_TOP) {
        const uint32_t m = heap_min_child(c, first, n, kmin, smin);
        ev = heap_get(c, m);
        uniform_event(ev);
        return m;
    }
    const int lane = lane_id();
    uint32_t i = first + (uint32_t)(lane & (K10S_HEAP_D - 1));
    int64_t k = 0x7FFFFFFFFFFFFFFFll;
    uint32_t sq = 0xFFFFFFFFu;
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    v4u lo = {0u, 0u, 0u, 0u};
    const __amdgpu_buffer_rsrc_t rs = heap_rsrc(c);
    if (lane < K10S_HEAP_D && i < n) {
        lo = __builtin_amdgcn_raw_buffer_load_b128(rs, heap_key_off(i), 0, 0);   // key halves only
        k = total_key(u2f(((uint64_t)lo[1] << 32) | lo[0]));
        sq = lo[2];
    }
    keymin_step<0>(k, sq, i);
    keymin_step<1>(k, sq, i);
    keymin_step<2>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 16) keymin_step<3>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 32) keymin_step<4>(k, sq, i);
    if constexpr (K10S_HEAP_D >= 64) keymin_step<5>(k, sq, i);
    const uint64_t klo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)k);
    const uint64_t khi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)k >> 32));
    kmin = (int64_t)(klo | (khi << 32));
    smin = (uint32_t)__builtin_amdgcn_readfirstlane((int)sq);
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
    const v4u hi = __builtin_amdgcn_raw_buffer_load_b128(rs, heap_pay_off(m), 0, 0);   // m's payload half
    const int src = (int)(m - first);   // the lane that loaded entry m's key half
    auto rl = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, src); };
    auto rf = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    ev.time = u2f(((uint64_t)rl(lo[1]) << 32) | rl(lo[0]));
    ev.seq = rl(lo[2]);
    const uint32_t ks = rl(lo[3]);
    ev.kind = (uint16_t)ks;
    ev.slot = (int16_t)(ks >> 16);
    ev.a = rf(hi[0]);
    ev.b = rf(hi[1]);
    ev.x = u2f(((uint64_t)rf(hi[3]) << 32) | rf(hi[2]));
    return m;
}
#define K10S_HEAP_POP_ATTR __attribute__((noinline))
#else
#define K10S_HEAP_POP_ATTR
#endif
K10S_HD K10S_HEAP_POP_ATTR void heap_pop(Ctx& c) {
    if (!K10S_FULL_WAVE(XG_HEAP_POP)) return;
    uint32_t n = uniform_u32(c.H().heap_size) - 1;
    c.H().heap_size = n;
    if (n == 0) return;
    HeapEv last = heap_get(c, n);
    [[maybe_unused]] uint32_t it = 0;
#if K10S_DEVICE
    bool have_last = false;
    int64_t kl = 0;
#else
    uniform_event(last);
    int64_t kl = total_key(last.time);
#endif
    uint32_t pos = 0;
    for (;;) {
        uint32_t first = K10S_HEAP_D * pos + 1;
        if (first >= n) break;
        if (K10S_LOOP_CAP(it, 12, XG_LOOP_HEAP_POP)) break;
        int64_t km;
        uint32_t sm;
#if K10S_DEVICE
        HeapEv child;
        uint32_t m = heap_min_child_ev(c, first, n, km, sm, child);
        if (!have_last) {
            uniform_event(last);
            kl = total_key(last.time);
            have_last = true;
        }
        if (!(km < kl || (km == kl && sm < last.seq))) break;
#else
        uint32_t m = heap_min_child(c, first, n, km, sm);
        if (!(km < kl || (km == kl && sm < last.seq))) break;
        HeapEv child = heap_get(c, m);
        uniform_event(child);
#endif
        heap_put(c, pos, child);
        if (pos == 0) c.H().heap_top = child;
        pos = m;
    }
#if K10S_DEVICE
    if (!have_last) uniform_event(last);
#endif
    heap_put(c, pos, last);
    if (pos == 0) c.H().heap_top = last;
}

// ---- Rust std BinaryHeap<QueuedPodInfo> (scheduler action queue) ------------------------------
// Ord: other.timestamp.total_cmp(&self.timestamp) => "a <= b" <=> b.ts <= a.ts (total order).
K10S_HD bool q_le(const QInfo& a, const QInfo& b) { return total_key(b.timestamp) <= total_key(a.timestamp); }

// Action-queue slot i: the top K10S_AQ_TOP positions in the working header, the rest in HBM.
// Loaded entries are wave-uniform by construction; saying so keeps the sift loops scalar.
K10S_HD QInfo aq_get(Ctx& c, uint32_t i) {
    QInfo q;
#if K10S_AQ_TOP
    if (i < K10S_AQ_TOP) q = c.H().aq_lds[i];
    else
#endif
    {
        q = c.V().aq()[i];
        K10S_HSTAT(HS_AQ_HBM_GET);
    }
#if K10S_DEVICE
    q.timestamp = uniform_f64(q.timestamp);
    q.initial = uniform_f64(q.initial);
    q.attempts = uniform_u32(q.attempts);
    q.pod = uniform_u32(q.pod);
#endif
    return q;
}
// The same slot as loaded, without making its fields wave-uniform: a sift moves whole entries but
// compares only timestamps, so the entries stay in VGPRs (stored back as loaded) and only the
// timestamp goes through readfirstlane (aq_ts) — 2 instead of 6 per entry read.
K10S_HD QInfo aq_raw(Ctx& c, uint32_t i) {
#if K10S_AQ_TOP
    if (i < K10S_AQ_TOP) return c.H().aq_lds[i];
#endif
    K10S_HSTAT(HS_AQ_HBM_GET);
    return c.V().aq()[i];
}
K10S_HD int64_t aq_ts(const QInfo& q) {
#if K10S_DEVICE
    return total_key(uniform_f64(q.timestamp));
#else
    return total_key(q.timestamp);
#endif
}
K10S_HD void aq_put(Ctx& c, uint32_t i, const QInfo& q) {
#if K10S_AQ_TOP
    if (i < K10S_AQ_TOP) {
        c.H().aq_lds[i] = q;
        return;
    }
#endif
    c.V().aq()[i] = q;
}

K10S_HD uint32_t aq_sift_up(Ctx& c, uint32_t start, uint32_t pos, const QInfo& elem) {
    [[maybe_unused]] uint32_t it = 0;
    const int64_t ke = aq_ts(elem);
    while (pos > start) {
        if (K10S_LOOP_CAP(it, 40, XG_LOOP_AQ_UP)) break;
        uint32_t parent = (pos - 1) / 2;
        const QInfo p = aq_raw(c, parent);
        if (ke >= aq_ts(p)) break;   // q_le(elem, p)
        aq_put(c, pos, p);
        pos = parent;
    }
    aq_put(c, pos, elem);
    return pos;
}
// Sorted mode (round 6).  While every push since the queue was last empty had a timestamp strictly
// above the previous push's, each push's sift_up stopped at once (queue.rs:29-33: elem <= parent),
// so the heap array is the pushes in order, strictly ascending — the Rust heap's array exactly.  The
// pops of a heap whose keys are distinct come out in ascending key order whatever its shape, so the
// i-th pop is the i-th entry: a push writes one entry and a pop reads one, with no sift.  Pops happen
// only in the scheduling cycle, which pops until the queue is empty and pushes nothing
// (scheduler.rs:261-330), so the front part its pops consume (aq_head) is never seen by a push, and
// aq_head returns to 0 when the queue empties.  The first push at or below the newest key leaves the
// mode: the array is the Rust heap's, and the usual sifts continue from it.  Ties (equal timestamps)
// always take the heap: their pop order depends on the heap's shape.  Measured on the host
// (one c3_backlog replica): after the arrivals end, 49 of 169 cycles and 48 % of the pops are in
// sorted mode; C3's arrivals come in equal-timestamp groups, so its cycles never are.
#ifndef K10S_AQ_SORTED
#define K10S_AQ_SORTED 1   // A/B knob: 0 = the heap always (round 5)
#endif
K10S_HELPER void aq_push(Ctx& c, const QInfo& q) {
    RepHdr& H = c.H();
    const uint32_t n = H.aq_size;
    if (n >= c.Ly().cap_aq) {
        fail(c, K10S_ERR_QUEUE_FULL);
        return;
    }
    const int64_t k = aq_ts(q);
    if (K10S_AQ_SORTED && (n == 0 || (H.aq_sorted && k > H.aq_last))) {   // (aq_head is 0 outside a cycle)
        aq_put(c, n, q);
        H.aq_sorted = 1;
        H.aq_last = k;
        H.aq_size = n + 1;
        return;
    }
    H.aq_sorted = 0;
    H.aq_size = n + 1;
    aq_sift_up(c, 0, n, q);
}
// (Round 3 tried reading the 3-level subtree under the walk's position in one round trip below the
// LDS levels into wave-uniform registers: C3 +0.6 %, backlog -2 to -4 % from the extra SGPRs live in
// the scheduling cycle, profiles/r03_k4_sflag_subtree_ab.json.  Round 4 keeps the subtree in VGPR
// lanes instead (below): backlog +8.7 %, C3 +0.2 %; the same pop out of line lost 1.5-2 % on C3,
// profiles/r04_h11_aq_batch_ab.json.)
K10S_HELPER QInfo aq_pop(Ctx& c) {
    K10S_HSTAT(HS_AQ_POP);
    if (c.H().aq_sorted) {   // sorted mode (aq_push): the front entry
        const uint32_t h = c.H().aq_head, n = c.H().aq_size - 1u;
        const QInfo q = aq_get(c, h);
        c.H().aq_size = n;
        c.H().aq_head = n ? h + 1u : 0u;
        return q;
    }
    const uint32_t end = --c.H().aq_size;
    QInfo item = aq_get(c, end);
    if (end == 0) return item;
    QInfo top = aq_get(c, 0);
    // sift_down_to_bottom(0) with `item` in the hole, then sift_up(0, pos)
    uint32_t pos = 0;
    uint32_t child = 1;
    [[maybe_unused]] uint32_t it = 0;
#if K10S_DEVICE
    // Three levels per memory round trip: lane r < 14 loads node r of the depth-3 subtree under pos
    // (level d = 1, 2, 3 at lanes 0-1, 2-5, 6-13; heap position ((pos + 1) << d) - 1 + j), the walk
    // compares the two candidate children of each level by readlane of their time keys, and every
    // lane whose entry moves up stores it at its new position in one masked store.  The walk itself
    // is the loop below, unchanged (same comparisons, same moves).
    {
        const uint32_t lane = (uint32_t)lane_id();
        const uint32_t d = lane < 2u ? 1u : lane < 6u ? 2u : 3u;
        const uint32_t j = lane + 2u - (1u << d);
        while (end >= 2 && child <= end - 2) {
            if (K10S_LOOP_CAP(it, 40, XG_LOOP_AQ_POP)) break;
            const uint32_t q = ((pos + 1u) << d) - 1u + j;
            QInfo x;
            x.timestamp = 0.0;
            x.initial = 0.0;
            x.attempts = 0;
            x.pod = 0;
            if (lane < 14u && q < end) x = aq_raw(c, q);
            const uint64_t kx = (uint64_t)total_key(x.timestamp);
            const uint32_t klo = (uint32_t)kx, khi = (uint32_t)(kx >> 32);
            uint32_t dest = 0xFFFFFFFFu;
            uint32_t jc = 0;   // the walk's node within its subtree level
            K10S_UNROLL
            for (uint32_t lv = 1; lv <= 3u; lv++) {
                if (!(child <= end - 2)) break;
                const uint32_t la = (1u << lv) - 2u + 2u * jc;
                const int64_t ka = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)khi, (int)la) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane((int)klo, (int)la));
                const int64_t kb = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)khi, (int)(la + 1u)) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane((int)klo, (int)(la + 1u)));
                const uint32_t pick = kb <= ka ? 1u : 0u;   // q_le(a, b): the right child
                dest = lane == la + pick ? pos : dest;
                pos = child + pick;
                child = 2u * pos + 1u;
                jc = 2u * jc + pick;
            }
            if (dest != 0xFFFFFFFFu) aq_put(c, dest, x);
        }
    }
#endif
    while (end >= 2 && child <= end - 2) {
        if (K10S_LOOP_CAP(it, 40, XG_LOOP_AQ_POP)) break;
        const QInfo a = aq_raw(c, child), b = aq_raw(c, child + 1);
        if (aq_ts(b) <= aq_ts(a)) {   // q_le(a, b): the right child
            aq_put(c, pos, b);
            child += 1;
        } else {
            aq_put(c, pos, a);
        }
        pos = child;
        child = 2 * pos + 1;
    }
    if (child == end - 1) {
        aq_put(c, pos, aq_raw(c, child));
        pos = child;
    }
    aq_sift_up(c, 0, pos, item);
    return top;
}

// ---- unschedulable_pods: BTreeMap<(insert_timestamp total_cmp, pod name)> as a sorted array -----
K10S_HD bool u_less(const QInfo& a, const QInfo& b) {
    int64_t ka = total_key(a.timestamp), kb = total_key(b.timestamp);
    return ka < kb || (ka == kb && a.pod < b.pod);
}
// The map's last key (RepHdr::uq_tail, round 6): a failed attempt's timestamp is its cycle's time
// plus the cycle's duration so far, above every entry already in the map, so the insert is an append.
// Knowing the tail's key, that append reads nothing (one dependent read per failed attempt before:
// the backlog fails about 4 attempts per placement).  A timestamp equal to the tail's, or an unknown
// tail (after the move / flush compactions), takes the walk below, which also restores the tail.
#ifndef K10S_UQ_TAIL
#define K10S_UQ_TAIL 1   // A/B knob: 0 = always the walk (round 5)
#endif
K10S_HELPER void uq_insert(Ctx& c, const QInfo& q) {
    if (c.H().uq_size >= c.Ly().cap_uq) {
        fail(c, K10S_ERR_QUEUE_FULL);
        return;
    }
    QInfo* d = c.V().uq();
    const int64_t kq = total_key(q.timestamp);
    uint32_t pos = c.H().uq_size++;
    if (K10S_UQ_TAIL && (pos == 0 || kq > c.H().uq_tail)) {
        d[pos] = q;   // strictly after every entry: no equal key to replace
        c.H().uq_tail = kq;
        return;
    }
    const uint32_t end = pos;   // the tail's position before this insert
    while (pos > 0) {  // timestamps are almost always >= the tail: short backward walk
        QInfo prev = d[pos - 1];
        if (!u_less(q, prev)) {
            if (prev.pod == q.pod && total_key(prev.timestamp) == total_key(q.timestamp)) {
                // BTreeMap::insert on an existing key replaces the value
                d[pos - 1] = q;
                for (uint32_t i = pos; i + 1 < c.H().uq_size; i++) d[i] = d[i + 1];
                c.H().uq_size--;
                return;   // (the tail's key is unchanged)
            }
            if (pos == end) c.H().uq_tail = kq;   // appended: q is the tail
            break;
        }
        if (pos == end) c.H().uq_tail = total_key(prev.timestamp);   // prev becomes the tail
        d[pos] = prev;
        pos--;
    }
    if (pos == 0 && end == 0) c.H().uq_tail = kq;
    d[pos] = q;
}

K10S_HD bool pod_in_s(const Ctx& c, uint32_t p) { return c.V().pod(p).sflag != 0; }

// move_pods_to_active_queue over a selection, in key order (scheduler.rs:174-185)
// mode 0: all (move_all_to_active_queue, 235-244); 1: flush (188-203, stay > 300 s);
// 2: freed-resources conditional (366-379); 3: inverted add-node conditional (396-405).
#if K10S_DEVICE
// move_all_to_active_queue on the device (scheduler.rs:235-244), out of line: the map's entries are
// read 64 at a time, one per lane, with their pods' cache flags (two memory round trips per 64
// entries instead of two per entry), then moved or kept in key order exactly as the loop below does
// (the entries of a batch come out of the lanes by readlane).  The backlog workload requeues the
// whole unschedulable map on every pod finish.
__device__ __attribute__((noinline)) void s_move_all_dev(Ctx& c) {
    QInfo* d = c.V().uq();
    const uint32_t n = uniform_u32(c.H().uq_size);
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t w = 0;
    uint64_t moved = 0;
    auto rl = [](uint32_t v, uint32_t j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j); };
    for (uint32_t base = 0; base < n; base += 64u) {
        const uint32_t cnt = n - base < 64u ? n - base : 64u;
        QInfo x;
        x.timestamp = 0.0;
        x.initial = 0.0;
        x.attempts = 0;
        x.pod = 0;
        uint32_t in_s = 0;
        if (lane < cnt) {
            x = d[base + lane];
            in_s = c.V().pod(x.pod).sflag;
        }
        const uint64_t live = __ballot(lane < cnt && in_s != 0);
        const uint64_t ts = f2u(x.timestamp), ti = f2u(x.initial);
        uint32_t j0 = 0;   // entries before j0 were moved by the bulk path
        {
            // Bulk append (round 6): when the action queue is empty or in sorted mode (aq_push) and this
            // batch's timestamps rise strictly, above the queue's newest, the live entries' pushes are
            // all sorted-mode appends: each lane writes its entry at the queue's end (rank among the
            // live lanes), the stale ones stay in the map in order.  Same array, counters and mode
            // as the pushes one by one.  The map is ordered by (timestamp, name), so equal
            // timestamps are adjacent: one compare with the lane below finds them.
            const uint32_t an = uniform_u32(c.H().aq_size);
            const bool srt = K10S_AQ_SORTED && (an == 0u || uniform_u32(c.H().aq_sorted) != 0u);
            const int64_t kx = total_key(x.timestamp);
            const uint32_t plo = (uint32_t)__shfl_up((int)(uint32_t)(uint64_t)kx, 1),
                           phi = (uint32_t)__shfl_up((int)(uint32_t)((uint64_t)kx >> 32), 1);
            const int64_t kp = lane == 0u ? (an == 0u ? (int64_t)0x8000000000000000ll
                                                       : (int64_t)uniform_u64((uint64_t)c.H().aq_last))
                                          : (int64_t)(((uint64_t)phi << 32) | plo);
            const bool rising = !(lane < cnt) || kx > kp;
            const uint32_t nl = (uint32_t)__popcll(live);
            if (srt && live && __ballot(!rising) == 0ull && an + nl <= c.Ly().cap_aq) {
                auto below = [&](uint64_t m) {
                    return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                };
                const bool mine = (live >> lane) & 1ull;
                QInfo q = x;
                q.attempts += 1u;
                if (mine) aq_put(c, an + below(live), q);
                const uint64_t stale = __ballot(lane < cnt) & ~live;
                if ((stale >> lane) & 1ull) d[w + below(stale)] = x;
                w += (uint32_t)__popcll(stale);
                const uint32_t hl = 63u - (uint32_t)__builtin_clzll(live);   // the newest moved entry
                c.H().aq_last = (int64_t)(((uint64_t)rl((uint32_t)((uint64_t)kx >> 32), hl) << 32) | rl((uint32_t)(uint64_t)kx, hl));
                c.H().aq_sorted = 1u;
                c.H().aq_size = an + nl;
                moved += nl;
                j0 = cnt;
            }
        }
        for (uint32_t j = j0; j < cnt; j++) {
            QInfo q;
            q.timestamp = u2f(((uint64_t)rl((uint32_t)(ts >> 32), j) << 32) | rl((uint32_t)ts, j));
            q.initial = u2f(((uint64_t)rl((uint32_t)(ti >> 32), j) << 32) | rl((uint32_t)ti, j));
            q.attempts = rl(x.attempts, j);
            q.pod = rl(x.pod, j);
            if ((live >> j) & 1u) {
                q.attempts += 1;
                aq_push(c, q);
                if (c.H().error_code) {
                    c.H().counters[K10S_C_REQUEUED] += moved;
                    return;
                }
                moved += 1;
            } else {
                d[w++] = q;  // a stale entry of a deleted pod stays
            }
        }
    }
    c.H().counters[K10S_C_REQUEUED] += moved;
    c.H().uq_size = w;
    c.H().uq_tail = 0x7FFFFFFFFFFFFFFFll;   // (the kept entries' last key: not tracked; uq_insert)
}
#endif
K10S_HELPER void s_move(Ctx& c, int mode, double t, uint32_t cpu, uint64_t ram) {
#if K10S_DEVICE
    if (mode == 0) {
        if (uniform_u32(c.H().uq_size) != 0) s_move_all_dev(c);
        return;
    }
#endif
    QInfo* d = c.V().uq();
    uint32_t n = c.H().uq_size;
    uint32_t w = 0;
    uint32_t fc = cpu;
    uint64_t fr = ram;
    if (mode >= 2) {
        // move_to_active_queue_if reads every entry's pod from the cache before moving any
        // (scheduler.rs:217-232): a stale entry panics with the queues untouched
        for (uint32_t i = 0; i < n; i++) {
            if (!pod_in_s(c, d[i].pod)) {
                fail(c, K10S_PANIC_MISSING_POD);
                return;
            }
        }
    }
    for (uint32_t i = 0; i < n; i++) {
        QInfo q = d[i];
        bool sel;
        if (mode == 0) {
            sel = true;
        } else if (mode == 1) {
            sel = (t - q.timestamp) > 5.0 * 60.0;
        } else {
            uint32_t rc = c.V().pod(q.pod).req_cpu;
            uint64_t rr = c.V().pod(q.pod).req_ram;
            if (rc <= fc && rr <= fr) {
                fc -= rc;
                fr -= rr;
                sel = (mode == 2);
            } else {
                sel = (mode == 3);
            }
        }
        if (sel && pod_in_s(c, q.pod)) {
            q.attempts += 1;
            aq_push(c, q);
            if (c.H().error_code) return;
            c.H().counters[K10S_C_REQUEUED] += 1;
            if (mode == 1) c.H().counters[K10S_C_FLUSHED] += 1;
        } else {
            d[w++] = q;  // kept (not selected, or stale entry of a deleted pod)
        }
    }
    c.H().uq_size = w;
    c.H().uq_tail = 0x7FFFFFFFFFFFFFFFll;   // (the kept entries' last key: not tracked; uq_insert)
}
K10S_HD void s_move_after_free(Ctx& c, uint32_t cpu, uint64_t ram) {
    if (c.P().enable_unscheduled_pods_conditional_move) s_move(c, 2, 0.0, cpu, ram);
    else s_move(c, 0, 0.0, 0, 0);
}

// ---- running pods of node components -----------------------------------------------------------
// A component's running_pods map (node_component.rs:33-47) is the set of pods whose run_slot is the
// component; only cancel_all_running_pods (95-112, node removal) iterates it, and nothing it does per
// pod depends on the order, so it is a lane-parallel sweep over run_slot (N_REMOVE_NODE) and a bind
// or finish touches only the pod's own line and the component's count.
// Remove running pod p (run_slot == slot, finish_seq == fs, the component's count srun and the
// pod's group g already loaded by the caller).
K10S_HD void run_remove_at(Ctx& c, uint32_t p, int32_t slot, uint32_t fs, int32_t srun, int32_t g) {
    PodState& P = c.V().pod(p);
    c.V().slot(slot).running = srun - 1;
    if (c.Ly().cap_gauge) {  // free_pod_requests (node_component.rs:88-91)
        c.V().g_cpu()[slot] += P.req_cpu;
        c.V().g_ram()[slot] += P.req_ram;
    }
    P.run_slot = -1;
    // cancels a pending finish event (dslab cancel_event) unless it is the one being handled: the
    // canceled event stays in the heap until popped (counted in stale_fin)
    if (fs != 0 && !(c.H().cur_kind == K10S_EV_N_POD_FINISHED && c.H().cur_seq == fs)) c.H().stale_fin += 1;
    P.finish_seq = 0;
    if (g >= 0) c.V().grp()[g].running -= 1;
}
K10S_HD void run_remove(Ctx& c, uint32_t p) {
    const PodState& P = c.V().pod(p);
    const int32_t slot = P.run_slot;
    run_remove_at(c, p, slot, P.finish_seq, c.V().slot(slot).running, c.S().pod_group[p]);
}

// ---- schedule_one: Fit filter + LeastAllocated score + argmax (the hot scan) -------------------
K10S_HD double la_score(uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr) {
    double cpu_score = (double)(uint32_t)(ac - rc) * 100.0 / (double)ac;
    double ram_score = (double)(uint64_t)(ar - rr) * 100.0 / (double)ar;
    return (cpu_score + ram_score) / 2.0;
}

// Returns K10S_SCHED_* and writes the chosen node index.  Wave-parallel over node indices (name
// order): each lane owns 4 consecutive nodes per 256-node step (one 16-B cpu load + two 16-B ram
// loads), keeps "score >= best" (the last maximum) over its nodes in ascending order, and the
// cross-lane (key, n) max reproduces the reference's left-to-right argmax.  The loads run
// K10S_SCAN_PIPE steps ahead of the arithmetic (software pipeline), so a wave keeps several
// 3 KiB steps in flight instead of waiting one memory round trip per step.
// Requires s_cpu / s_ram 16-B aligned and readable up to the next multiple of 4 nodes (engine
// sections are 256-B padded; the unit surface's rows are node_stride (multiple of 64) long).
// K10S_SCAN_PIPE: the unit-surface kernel (k10s_schedule_kernel, HBM-bound: 1 measured best);
// K10S_LOOP_SCAN_PIPE: the scans inside the event loop (0 measured +1.2 % on C3 and +1.7 % on the
// backlog workload over 1 with the cycle out of line, profiles/r02_v5_knobs_ab.json).
#ifndef K10S_LOOP_SCAN_PIPE
#define K10S_LOOP_SCAN_PIPE 0
#endif
#ifndef K10S_SCAN_PIPE
#define K10S_SCAN_PIPE 1
#endif
K10S_HD void scan_node(uint32_t n, uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr, double weight, int32_t& first,
                       uint64_t& best_key, int32_t& best_n) {
    if (rc <= ac && rr <= ar) {
        if ((int32_t)n < first) first = (int32_t)n;
        double s = 0.0 + la_score(ac, ar, rc, rr) * weight;
        if (!is_nan(s)) {
            uint64_t k = score_key(s);
            if (k >= best_key) {
                best_key = k;
                best_n = (int32_t)n;
            }
        }
    }
}

#if K10S_DEVICE
struct ScanGrp {            // one lane's 4 consecutive nodes of a 256-node step, as loaded
    uint64_t pw;            // the presence word holding them
    uint4 cv;
    ulonglong2 r01, r23;
};
// Unconditional loads: a lane past the end re-reads nodes 0..3 (n_nodes >= 1; valid and cached) and grp_bits() masks it out, so no branch and no zero fill sits
// between the load and its use.
K10S_D ScanGrp scan_load(const uint32_t* s_cpu, const uint64_t* s_ram, const uint64_t* present, uint32_t n_nodes,
                         uint32_t n0) {
    const uint32_t a = n0 < n_nodes ? n0 : 0u;
    ScanGrp g;
    g.pw = present[a >> 6];
    g.cv = *reinterpret_cast<const uint4*>(s_cpu + a);
    g.r01 = *reinterpret_cast<const ulonglong2*>(s_ram + a);
    g.r23 = *reinterpret_cast<const ulonglong2*>(s_ram + a + 2);
    return g;
}
// The event loop's screened scan (rc > 0): absent nodes hold (0, 0) in the cache (S_REMOVE_NODE,
// init_replica), so Fit alone excludes them and the presence word is not read.
K10S_D ScanGrp scan_load_np(const uint32_t* s_cpu, const uint64_t* s_ram, uint32_t n_nodes, uint32_t n0) {
    const uint32_t a = n0 < n_nodes ? n0 : 0u;
    ScanGrp g;
    g.pw = ~0ull;
    g.cv = *reinterpret_cast<const uint4*>(s_cpu + a);
    g.r01 = *reinterpret_cast<const ulonglong2*>(s_ram + a);
    g.r23 = *reinterpret_cast<const ulonglong2*>(s_ram + a + 2);
    return g;
}
// The packed node cache (nc_*): a lane's 4 consecutive u64 entries (two 16-B loads, 32 B instead of
// 48), split into the same (cpu, ram) group the wide loads give.  PRES: read the presence word.
K10S_D ScanGrp scan_load_pk(const uint64_t* s_node, const uint64_t* present, uint32_t n_nodes, uint32_t n0,
                            bool pres) {
    const uint32_t a = n0 < n_nodes ? n0 : 0u;
    ScanGrp g;
    g.pw = pres ? present[a >> 6] : ~0ull;
    const ulonglong2 x01 = *reinterpret_cast<const ulonglong2*>(s_node + a);
    const ulonglong2 x23 = *reinterpret_cast<const ulonglong2*>(s_node + a + 2);
    g.cv.x = (uint32_t)(x01.x >> K10S_PK_SHIFT);
    g.cv.y = (uint32_t)(x01.y >> K10S_PK_SHIFT);
    g.cv.z = (uint32_t)(x23.x >> K10S_PK_SHIFT);
    g.cv.w = (uint32_t)(x23.y >> K10S_PK_SHIFT);
    g.r01.x = x01.x & K10S_PK_RAM;
    g.r01.y = x01.y & K10S_PK_RAM;
    g.r23.x = x23.x & K10S_PK_RAM;
    g.r23.y = x23.y & K10S_PK_RAM;
    return g;
}
// A whole group inside the node range (no clamp, no presence word).
K10S_D ScanGrp scan_load_pk_full(const uint64_t* s_node, uint32_t n0) {
    ScanGrp g;
    g.pw = ~0ull;
    const ulonglong2 x01 = *reinterpret_cast<const ulonglong2*>(s_node + n0);
    const ulonglong2 x23 = *reinterpret_cast<const ulonglong2*>(s_node + n0 + 2);
    g.cv.x = (uint32_t)(x01.x >> K10S_PK_SHIFT);
    g.cv.y = (uint32_t)(x01.y >> K10S_PK_SHIFT);
    g.cv.z = (uint32_t)(x23.x >> K10S_PK_SHIFT);
    g.cv.w = (uint32_t)(x23.y >> K10S_PK_SHIFT);
    g.r01.x = x01.x & K10S_PK_RAM;
    g.r01.y = x01.y & K10S_PK_RAM;
    g.r23.x = x23.x & K10S_PK_RAM;
    g.r23.y = x23.y & K10S_PK_RAM;
    return g;
}
// PK: s_ram is the packed node array (s_cpu unused)
template <bool PK>
K10S_D ScanGrp scan_load_x(const uint32_t* s_cpu, const uint64_t* s_ram, const uint64_t* present, uint32_t n_nodes,
                           uint32_t n0) {
    return PK ? scan_load_pk(s_ram, present, n_nodes, n0, true) : scan_load(s_cpu, s_ram, present, n_nodes, n0);
}
K10S_D uint32_t grp_bits(const ScanGrp& g, uint32_t n0, uint32_t n_nodes) {
    if (n0 >= n_nodes) return 0;
    const uint32_t valid = n_nodes - n0;
    return (uint32_t)(g.pw >> (n0 & 63)) & (valid >= 4 ? 0xFu : ((1u << valid) - 1u));
}
// Device form of la_score's two quotients: the same operations the compiler emits for an IEEE f64
// division (v_rcp_f64, two Newton steps, q = x·r, one remainder correction), minus the
// v_div_scale / v_div_fixup pair.  Those only change anything when an operand is 0, inf/NaN, near
// the denormal range or 2^±768 apart; here x = 100·(a − r) and y = a are integers in [0, 2^71) with
// x/y in [0, 100], so scale is the identity (and div_fmas a plain fma), and the result is bit-for-
// bit the correctly rounded quotient.  The one special case that occurs, 0/0 (a == r == 0), gives
// NaN through rcp(0) = inf, as the IEEE division does (plugin.rs:52-63).
K10S_D double div_rn(double x, double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = x * r;
    const double rem = __builtin_fma(-y, q, x);
    return __builtin_fma(rem, r, q);
}
// u64 -> f64 with one rounding (hi·2^32 is exact; the fma rounds hi·2^32 + lo once), = Rust `as f64`.
// (The high word's u32 -> f64 is written as the instruction itself: as C the compiler re-forms the
// u64 conversion and adds a dead 0·2^32 term.)
K10S_D double u64_f64(uint64_t v) {
    const uint2 w = __builtin_bit_cast(uint2, v);
    double hi;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hi) : "v"(w.y));
    return __builtin_fma(hi, 4294967296.0, (double)w.x);
}
// la_score on the device (plugin.rs:52-63), bit-identical to la_score.  Also the elementwise
// ScorePlugin surface k10s_score_batch.
K10S_D double la_score_d(uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr) {
    const double cs = div_rn((double)(ac - rc) * 100.0, (double)ac);
    const double rs = div_rn(u64_f64(ar - rr) * 100.0, u64_f64(ar));
    return (cs + rs) * 0.5;  // (c + r) / 2.0, exact halving
}
// scan_node on the device: the score stays a double and the lane max is an f64 compare.  The
// score is never -0.0 (a +0 quotient sum, or 0.0 + s·w), so for non-NaN scores ">=" on doubles is
// the score_key order, NaN never compares true (= "NaN is never selected"), and -inf as the start
// value accepts the first non-NaN score like score_key's 0.  W1: weight == 1.0, where 0.0 + s·1.0
// is the identity on scores >= +0 and NaN.
template <bool W1, bool TF>
K10S_D void scan_node_d(uint32_t n, bool present, uint32_t ac, uint64_t ar, uint32_t rc, uint64_t rr, double frc,
                        double frr, double weight, int32_t& first, double& best_s, int32_t& best_n) {
    if (rc <= ac && rr <= ar && present) {
        if (TF) first = (int32_t)n < first ? (int32_t)n : first;
        const double fac = (double)ac;
        const double cs = div_rn((fac - frc) * 100.0, fac);
        const uint2 w = __builtin_bit_cast(uint2, ar);
        const double far = u64_f64(ar);
        double dr = far - frr;
        if (__builtin_expect(w.y >= (1u << 21), 0)) dr = u64_f64(ar - rr);
        double s = (cs + div_rn(dr * 100.0, far)) * 0.5;
        if (!W1) s = 0.0 + s * weight;
        if (s >= best_s) {
            best_s = s;
            best_n = (int32_t)n;
        }
    }
}
template <bool W1, bool TF>
K10S_D void scan_grp(const ScanGrp& g, uint32_t n0, uint32_t n_nodes, uint32_t rc, uint64_t rr, double frc,
                     double frr, double weight, int32_t& first, double& best_s, int32_t& best_n) {
    const uint32_t bits = grp_bits(g, n0, n_nodes);
    if (bits) {
        scan_node_d<W1, TF>(n0, bits & 1u, g.cv.x, g.r01.x, rc, rr, frc, frr, weight, first, best_s, best_n);
        scan_node_d<W1, TF>(n0 + 1, bits & 2u, g.cv.y, g.r01.y, rc, rr, frc, frr, weight, first, best_s, best_n);
        scan_node_d<W1, TF>(n0 + 2, bits & 4u, g.cv.z, g.r23.x, rc, rr, frc, frr, weight, first, best_s, best_n);
        scan_node_d<W1, TF>(n0 + 3, bits & 8u, g.cv.w, g.r23.y, rc, rr, frc, frr, weight, first, best_s, best_n);
    }
}
template <bool W1, bool TF, int PIPE, bool PK = false>
K10S_D void scan_lanes(const uint32_t* s_cpu, const uint64_t* s_ram, const uint64_t* present, uint32_t n_nodes,
                       uint32_t rc, uint64_t rr, double weight, int32_t& first, double& best_s, int32_t& best_n) {
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    // the pod's request is wave-uniform: keep it (and its f64 forms) in SGPRs, out of the VGPR budget
    rc = uniform_u32(rc);
    rr = uniform_u64(rr);
    const double frc = uniform_f64((double)rc), frr = uniform_f64(u64_f64(rr));
    if (n_nodes == 0) return;
    // Software pipeline: loads run PIPE steps (of 256 nodes) ahead of the arithmetic.
    ScanGrp g[PIPE + 1];
#pragma unroll
    for (int i = 0; i < PIPE; i++) g[i] = scan_load_x<PK>(s_cpu, s_ram, present, n_nodes, 256u * i + l4);
    for (uint32_t base = 0; base < n_nodes; base += 256) {
        g[PIPE] = scan_load_x<PK>(s_cpu, s_ram, present, n_nodes, base + 256u * PIPE + l4);
        scan_grp<W1, TF>(g[0], base + l4, n_nodes, rc, rr, frc, frr, weight, first, best_s, best_n);
#pragma unroll
        for (int i = 0; i < PIPE; i++) g[i] = g[i + 1];
    }
}
#endif

// ---- screened scan (weight 1.0, rc > 0, rr > 0: the event loop and the unit surface) -----------
// With u = rc/A + rr/R, a fitting node's LeastAllocated score is 100 − 50·u (plugin.rs:52-63), so
// the argmax is the u minimum.  Each lane keeps lu, the smallest u among the nodes it scored, and
// after every 256-node step the wave takes thr = min lu: some scored node y has u(y) <= thr
// (within f32 rounding).  A later node x whose single-precision, division-free test
//     rc·R + rr·A  >  A·R·(thr + eps)            (scan_screen, eps = 1e-5)
// holds has, in exact arithmetic, u(x) > u(y) + 9.9e-6 − 36·2^-24 > u(y) + 7e-6, so its exact
// score is more than 3e-4 below y's and its computed f64 score is strictly below y's computed
// score (each within 3.4e-14 of exact): x can never be the (score, last index) argmax, and is
// not scored.  Every other fitting node is scored exactly as in scan_node_d — except a node with
// exactly the lane's best allocatables, which has exactly its score and just takes the index.
// f32 ranges: A·R < 2^96, no overflow; all operands >= 1, no denormals.  The bound is checked at
// and around the threshold by tests/test_scan_screen.py through the host form of this test.
#define K10S_SCREEN_EPS 1e-5f
K10S_HD bool scan_screen(uint32_t ac, uint64_t ar, float fa, float fr, float T) {
    const float fA = (float)ac;
    const float fR = __builtin_fmaf((float)(uint32_t)(ar >> 32), 4294967296.0f, (float)(uint32_t)ar);
    return __builtin_fmaf(fa, fR, fr * fA) > fA * fR * T;
}
// u of a scored node from its exact score: (100 − s)/50, rounded to f32.
K10S_HD float screen_u(double s) { return (float)((100.0 - s) * 0.02); }

#if K10S_DEVICE
// The event loop's fast-path scans screen (+2.0 % at C3 once the scheduling cycle runs out of line
// with its own registers, profiles/r02_v6_scan_screen_ab.json; inlined into the event loop its state
// spilled inside the scan, r02_v3_scan_experiments_ab.json), and so does the unit surface
// (k10s_schedule_kernel: scoring every node exactly, two f64 divisions each, made it VALU-bound below
// the HBM roofline, r02_v27_unit_screen.json).
// scan_lanes_screen evaluates the screen of a lane's 4 nodes first (screen_grp), then scores the
// remaining ones in order (score_node_exact): the conversions are single v_cvt_f32_u32 each, the
// products run 2 nodes per v_pk_mul_f32 / v_pk_fma_f32, and no exec-mask branch separates the 4
// nodes (round 2 tested and scored node by node: -59 VALU per event, +4.9 % at C3).
typedef float f32x2 __attribute__((ext_vector_type(2)));
K10S_D float cvt_f32_u32(uint32_t v) {   // (float)v, correctly rounded, as the one instruction
    float f;
    asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"(v));
    return f;
}
// nk: node k of the group is present, fits, and is not ruled out by the screen (scan_screen).  Kept
// as four bools, the compares' lane masks combine on the scalar unit and gate the exact scores
// directly; packed into a 4-bit integer they cost a v_cndmask / v_or / v_cmp each per node.
struct Need4 {
    bool n0, n1, n2, n3;
};
// The screen alone: nk is false when scan_screen rules node k out (A: cpu, H/L: ram's high and low
// words, each converted to f32 exactly as one instruction).
K10S_D Need4 screen_keep(f32x2 A01, f32x2 A23, f32x2 H01, f32x2 H23, f32x2 L01, f32x2 L23, float fa, float fr, float T) {
    const f32x2 two32 = {4294967296.0f, 4294967296.0f};
    const f32x2 R01 = __builtin_elementwise_fma(H01, two32, L01), R23 = __builtin_elementwise_fma(H23, two32, L23);
    const f32x2 va = {fa, fa}, vr = {fr, fr}, vT = {T, T};
    const f32x2 l01 = __builtin_elementwise_fma(va, R01, vr * A01), l23 = __builtin_elementwise_fma(va, R23, vr * A23);
    const f32x2 r01 = (A01 * R01) * vT, r23 = (A23 * R23) * vT;
    return {!(l01.x > r01.x), !(l01.y > r01.y), !(l23.x > r23.x), !(l23.y > r23.y)};
}
K10S_D Need4 screen_grp(const ScanGrp& g, uint32_t bits, uint32_t rc, uint64_t rr, float fa, float fr, float T) {
    const bool f0 = (bits & 1u) && rc <= g.cv.x && rr <= g.r01.x;
    const bool f1 = (bits & 2u) && rc <= g.cv.y && rr <= g.r01.y;
    const bool f2 = (bits & 4u) && rc <= g.cv.z && rr <= g.r23.x;
    const bool f3 = (bits & 8u) && rc <= g.cv.w && rr <= g.r23.y;
    const f32x2 A01 = {cvt_f32_u32(g.cv.x), cvt_f32_u32(g.cv.y)};
    const f32x2 A23 = {cvt_f32_u32(g.cv.z), cvt_f32_u32(g.cv.w)};
    const f32x2 H01 = {cvt_f32_u32((uint32_t)(g.r01.x >> 32)), cvt_f32_u32((uint32_t)(g.r01.y >> 32))};
    const f32x2 H23 = {cvt_f32_u32((uint32_t)(g.r23.x >> 32)), cvt_f32_u32((uint32_t)(g.r23.y >> 32))};
    const f32x2 L01 = {cvt_f32_u32((uint32_t)g.r01.x), cvt_f32_u32((uint32_t)g.r01.y)};
    const f32x2 L23 = {cvt_f32_u32((uint32_t)g.r23.x), cvt_f32_u32((uint32_t)g.r23.y)};
    const Need4 k = screen_keep(A01, A23, H01, H23, L01, L23, fa, fr, T);
    return {f0 && k.n0, f1 && k.n1, f2 && k.n2, f3 && k.n3};
}
// The packed cache's whole-block path: a lane's 4 entries as loaded, (lo, hi) words each (cpu =
// hi >> 8, ram = (hi & 0xff)·2^32 + lo for K10S_PK_SHIFT 40).  The screen runs first on the raw
// words — the ram's high byte converts with v_cvt_f32_ubyte0, so nothing is masked — and Fit only
// for the nodes it keeps, which are few once the wave has a threshold: a node that does not fit
// has u = rc/A + rr/R > 1, far above any scored node's.  Kept-and-fitting is exactly screen_grp's
// set, so the same nodes are scored in the same order.
static_assert(K10S_PK_SHIFT == 40, "pk_* helpers assume the ram's high word is the entry's low byte of hi");
struct PkGrp {
    uint2 w0, w1, w2, w3;
};
K10S_D PkGrp pk_load_full(const uint64_t* s_node, uint32_t n0) {
    const uint4 a = *reinterpret_cast<const uint4*>(s_node + n0);
    const uint4 b = *reinterpret_cast<const uint4*>(s_node + n0 + 2);
    return {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
}
K10S_D float cvt_f32_ubyte0(uint32_t v) {   // (float)(v & 0xff), as the one instruction
    float f;
    asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(v));
    return f;
}
K10S_D uint32_t pk_cpu(uint2 w) { return w.y >> (K10S_PK_SHIFT - 32); }
K10S_D uint64_t pk_ram(uint2 w) { return ((uint64_t)(w.y & 0xffu) << 32) | w.x; }
K10S_D Need4 screen_pk(const PkGrp& g, float fa, float fr, float T) {
    const f32x2 A01 = {cvt_f32_u32(pk_cpu(g.w0)), cvt_f32_u32(pk_cpu(g.w1))};
    const f32x2 A23 = {cvt_f32_u32(pk_cpu(g.w2)), cvt_f32_u32(pk_cpu(g.w3))};
    const f32x2 H01 = {cvt_f32_ubyte0(g.w0.y), cvt_f32_ubyte0(g.w1.y)};
    const f32x2 H23 = {cvt_f32_ubyte0(g.w2.y), cvt_f32_ubyte0(g.w3.y)};
    const f32x2 L01 = {cvt_f32_u32(g.w0.x), cvt_f32_u32(g.w1.x)};
    const f32x2 L23 = {cvt_f32_u32(g.w2.x), cvt_f32_u32(g.w3.x)};
    return screen_keep(A01, A23, H01, H23, L01, L23, fa, fr, T);
}
// The exact LeastAllocated score of a fitting node (scan_node_d's arithmetic; frc, frr: the request
// as f64).
K10S_D double la_exact(uint32_t ac, uint64_t ar, uint64_t rr, double frc, double frr) {
    const double fac = (double)ac;
    const double cs = div_rn((fac - frc) * 100.0, fac);
    const uint2 w = __builtin_bit_cast(uint2, ar);
    const double far = u64_f64(ar);
    double dr = far - frr;
    if (__builtin_expect(w.y >= (1u << 21), 0)) dr = u64_f64(ar - rr);
    return (cs + div_rn(dr * 100.0, far)) * 0.5;
}
// A fitting node the screen did not rule out: the lane best's allocatables take the index (same
// score), anything else is scored exactly (as scan_node_d).
K10S_D void score_node_exact(uint32_t n, uint32_t ac, uint64_t ar, uint64_t rr, double frc, double frr, double& best_s,
                             int32_t& best_n, uint32_t& la, uint64_t& lr, float& lu) {
    if (ac == la && ar == lr) {
        best_n = (int32_t)n;
        return;
    }
    const double s = la_exact(ac, ar, rr, frc, frr);
    if (s >= best_s) {
        best_s = s;
        best_n = (int32_t)n;
        la = ac;
        lr = ar;
    }
    const float u = screen_u(s);
    lu = u < lu ? u : lu;
}
template <int S>
K10S_D float minf_step(float v) {
    uint32_t a, b;
    xpair<S>(__builtin_bit_cast(uint32_t, v), a, b);
    const float fa = __builtin_bit_cast(float, a), fb = __builtin_bit_cast(float, b);
    return fa < fb ? fa : fb;
}
K10S_D float wave_min_f32(float v) {
    v = minf_step<0>(v); v = minf_step<1>(v); v = minf_step<2>(v);
    v = minf_step<3>(v); v = minf_step<4>(v); v = minf_step<5>(v);
    return v;
}
// NP: the event loop's own node cache (absent nodes hold (0, 0), so Fit alone excludes them with
// rc > 0: no presence words read, r02_v10_presence_split_ab.json); the unit surface's caller-owned
// buffers keep their presence bitmap.
#define SCREEN_LOAD(c, r, p, n, n0) \
    (PK ? scan_load_pk(r, p, n, n0, !NP) : (NP ? scan_load_np(c, r, n, n0) : scan_load(c, r, p, n, n0)))
template <int PIPE, bool NP = true, bool PK = false>
K10S_D void scan_lanes_screen(const uint32_t* s_cpu, const uint64_t* s_ram, const uint64_t* present, uint32_t n_nodes,
                              uint32_t rc, uint64_t rr, double& best_s, int32_t& best_n) {
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    rc = uniform_u32(rc);
    rr = uniform_u64(rr);
    const double frc = uniform_f64((double)rc), frr = uniform_f64(u64_f64(rr));
    const float fa = (float)rc;
    const float fr = __builtin_fmaf((float)(uint32_t)(rr >> 32), 4294967296.0f, (float)(uint32_t)rr);
    if (n_nodes == 0) return;
    uint32_t la = 0;   // the lane best's allocatables (0: none; a fitting node has both >= 1)
    uint64_t lr = 0;
    float lu = __builtin_inff();
    float T = __builtin_inff();  // thr + eps: +inf screens nothing out (the first step)
    // one 256-node step of a lane's group g at n0 (screen, exact scores, threshold)
    auto step = [&](const ScanGrp& g, uint32_t n0, auto full) {
        const uint32_t bits = decltype(full)::value ? 0xFu : grp_bits(g, n0, n_nodes);
        const Need4 need = screen_grp(g, bits, rc, rr, fa, fr, T);
        const bool any = need.n0 | need.n1 | need.n2 | need.n3;
        if (any) {
            if (need.n0) score_node_exact(n0, g.cv.x, g.r01.x, rr, frc, frr, best_s, best_n, la, lr, lu);
            if (need.n1) score_node_exact(n0 + 1, g.cv.y, g.r01.y, rr, frc, frr, best_s, best_n, la, lr, lu);
            if (need.n2) score_node_exact(n0 + 2, g.cv.z, g.r23.x, rr, frc, frr, best_s, best_n, la, lr, lu);
            if (need.n3) score_node_exact(n0 + 3, g.cv.w, g.r23.y, rr, frc, frr, best_s, best_n, la, lr, lu);
        }
        if (__ballot(any)) {
            const float thr = __builtin_bit_cast(float, uniform_u32(__builtin_bit_cast(uint32_t, wave_min_f32(lu))));
            T = thr + K10S_SCREEN_EPS;
        }
    };
    // Packed node cache, no load pipeline: the loads of two 256-node steps (32 B per lane each) are
    // issued together, so a 4,096-node scan waits 8 memory round trips, not 16 (+2.4 %,
    // r03_s4_knobs_ab.json); a lane still visits its nodes in ascending order.  In the event loop
    // (no presence words) whole 512-node blocks load from unclamped addresses and screen all 4 nodes
    // of a lane group without a validity mask; only the last, partial block builds one.
    if (PK && PIPE == 0) {
        uint32_t base = 0;
        if (NP) {
            // one 256-node step on the raw packed words (screen_pk; Fit after the screen)
            auto step_pk = [&](const PkGrp& g, uint32_t n0) {
                const Need4 keep = screen_pk(g, fa, fr, T);
                bool scored = false;
                if (keep.n0 | keep.n1 | keep.n2 | keep.n3) {
                    auto one = [&](bool kept, uint2 w, uint32_t n) {
                        const uint32_t ac = pk_cpu(w);
                        const uint64_t ar = pk_ram(w);
                        if (kept && rc <= ac && rr <= ar) {
                            score_node_exact(n, ac, ar, rr, frc, frr, best_s, best_n, la, lr, lu);
                            scored = true;
                        }
                    };
                    one(keep.n0, g.w0, n0);
                    one(keep.n1, g.w1, n0 + 1);
                    one(keep.n2, g.w2, n0 + 2);
                    one(keep.n3, g.w3, n0 + 3);
                }
                if (__ballot(scored)) {
                    const float thr = __builtin_bit_cast(float, uniform_u32(__builtin_bit_cast(uint32_t, wave_min_f32(lu))));
                    T = thr + K10S_SCREEN_EPS;
                }
            };
            for (; base + 512u <= n_nodes; base += 512) {
                const PkGrp g0 = pk_load_full(s_ram, base + l4);
                const PkGrp g1 = pk_load_full(s_ram, base + 256u + l4);
                step_pk(g0, base + l4);
                step_pk(g1, base + 256u + l4);
            }
        }
        for (; base < n_nodes; base += 512) {
            const ScanGrp g0 = SCREEN_LOAD(s_cpu, s_ram, present, n_nodes, base + l4);
            const ScanGrp g1 = SCREEN_LOAD(s_cpu, s_ram, present, n_nodes, base + 256u + l4);
            step(g0, base + l4, std::false_type());
            step(g1, base + 256u + l4, std::false_type());
        }
        return;
    }
    ScanGrp g[PIPE + 1];
#pragma unroll
    for (int i = 0; i < PIPE; i++) g[i] = SCREEN_LOAD(s_cpu, s_ram, present, n_nodes, 256u * i + l4);
    for (uint32_t base = 0; base < n_nodes; base += 256) {
        g[PIPE] = SCREEN_LOAD(s_cpu, s_ram, present, n_nodes, base + 256u * PIPE + l4);
        const uint32_t n0 = base + l4;
        // (thr only moves when some lane scored a node exactly this step: the 6-step wave reduction
        // is skipped otherwise, T is then exactly what it would give)
        step(g[0], n0, std::false_type());
#pragma unroll
        for (int i = 0; i < PIPE; i++) g[i] = g[i + 1];
    }
}
#endif

// LOOP: the event loop's scans (K10S_LOOP_SCAN_PIPE) rather than the unit surface's (K10S_SCAN_PIPE).
// PK: s_ram is the packed node array (nc_*), s_cpu is not read.
template <bool LOOP = false, bool PK = false>
K10S_HD int schedule_scan(const uint32_t* s_cpu, const uint64_t* s_ram, const uint64_t* present, uint32_t n_nodes,
                          uint32_t rc, uint64_t rr, double weight, int32_t* chosen) {
    uint64_t best_key = 0;
    int32_t best_n = -1;
    int32_t first = 0x7fffffff;
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_SCHEDULE_SCAN)) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    double best_s = -__builtin_inf();
    if (weight == 1.0 && rc > 0 && rr > 0) {
        // A fitting node has alloc >= request > 0 in both resources, so neither term is 0/0 and every
        // score is a finite number >= 0: filtered[0] is never NaN, "some node fits" <=> best_n >= 0,
        // and neither filtered[0] nor its re-scored value is needed (kube_scheduler.rs:140-148).
        if (LOOP)
            scan_lanes_screen<K10S_LOOP_SCAN_PIPE, true, PK>(s_cpu, s_ram, present, n_nodes, rc, rr, best_s, best_n);
        else
            scan_lanes_screen<K10S_SCAN_PIPE, false, PK>(s_cpu, s_ram, present, n_nodes, rc, rr, best_s, best_n);
        best_key = best_n >= 0 ? score_key(best_s) : 0;
        wave_argmax(best_key, best_n);
        if (best_n < 0) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
        *chosen = best_n;
        return K10S_SCHED_OK;
    }
    constexpr int P = LOOP ? K10S_LOOP_SCAN_PIPE : K10S_SCAN_PIPE;
    if (weight == 1.0) scan_lanes<true, true, P, PK>(s_cpu, s_ram, present, n_nodes, rc, rr, weight, first, best_s, best_n);
    else scan_lanes<false, true, P, PK>(s_cpu, s_ram, present, n_nodes, rc, rr, weight, first, best_s, best_n);
    best_key = best_n >= 0 ? score_key(best_s) : 0;
#else
    for (uint32_t n = 0; n < n_nodes; n++) {
        if (!((present[n >> 6] >> (n & 63)) & 1ull)) continue;
        const NcEnt v = PK ? nc_unpack(s_ram[n]) : NcEnt{s_cpu[n], s_ram[n]};
        scan_node(n, v.cpu, v.ram, rc, rr, weight, first, best_key, best_n);
    }
#endif
    first = wave_min_i32(first);
    wave_argmax(best_key, best_n);
    if (first == 0x7fffffff) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    // kube_scheduler.rs:140-148: start from filtered[0]; if its score is NaN nothing replaces it
    const NcEnt v0 = PK ? nc_unpack(s_ram[first]) : NcEnt{s_cpu[first], s_ram[first]};
    double s0 = 0.0 + la_score(v0.cpu, v0.ram, rc, rr) * weight;
    *chosen = is_nan(s0) ? first : best_n;
    return K10S_SCHED_OK;
}

// ---- per-block fronts of the packed node cache (round 6) -----------------------------------------
// Which nodes can be schedule_one's answer at all.  With weight 1.0 and both requests > 0 the
// LeastAllocated score is monotone in (cpu, ram) (correctly rounded quotients of exactly represented
// integers: schedule_scan_pruned's argument) and Fit is too, so a node n is never the answer when a
// later node m > n (name order) has at least as much of both: m fits whenever n does, scores at least
// as much, and wins a tie (the last maximum, kube_scheduler.rs:140-148).  The answer is therefore in
// the index-aware front {n : no m > n with cpu_m >= cpu_n and ram_m >= ram_n}, and within any block
// of nodes in the block's own front.  At C3 the whole cache's front holds 40 of 4,096 nodes and a
// 64-node block's 3.9 on average (tools/prune_study.py): identical empty nodes collapse to their
// last one, and a loaded node below an empty one of its type never wins.
// The engine keeps, per 64-node block (<= 64 blocks, N <= 4,096), its front's entries and node
// offsets (K10S_FR_K slots; a block with more is scanned whole: fr_over), rebuilt lazily: every change
// of an entry (reserve, release, add, remove) marks its block in fr_dirty, and the next scan rebuilds
// the marked blocks first (four per memory round trip).  A fast-path attempt then reads K10S_FR_K
// slots per block (512 B per 64 blocks... 4 KB at C3) instead of the whole cache (32 KB), scores them
// like the screened scan (the first slot exactly, the rest screened against the wave's threshold),
// and takes the wave's (score, index) maximum.  The result is the full scan's by the argument above;
// entries read = slots + rebuilt and overflowing blocks' nodes.
// (K10S_FR_K, the front slots per block: k10s_state.h)
#ifndef K10S_FRONT_COMPACT
#define K10S_FRONT_COMPACT 1   // A/B knob: 0 = one exact-scoring branch per slot any lane kept
#endif
#if K10S_DEVICE
K10S_D uint64_t readlane_u64(uint64_t v, uint32_t j) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)j) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)j);
}
// Block b's front from its entries (lane i holds node 64b + i, 0 past the end): the highest lane that
// no processed front lane dominates is itself in the front (every lane above it is in the front or
// dominated by a front lane above it, which would dominate it too); it then marks the lanes below it
// that it dominates.  One iteration per front node.  Returns the front's size.
K10S_D uint32_t fr_block(uint64_t* fv, uint8_t* fi, uint32_t b, uint64_t x) {
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t cpu = (uint32_t)(x >> K10S_PK_SHIFT);
    const uint64_t ram = x & K10S_PK_RAM;
    bool dom = x == 0;   // an absent node holds (0, 0): it fits no request with cpu > 0
    uint64_t front = 0;
    for (;;) {
        const uint64_t cand = __ballot(!dom) & ~front;
        if (cand == 0) break;
        const uint32_t j = 63u - (uint32_t)__builtin_clzll(cand);
        front |= 1ull << j;
        const uint64_t xj = readlane_u64(x, j);
        dom = dom || (lane < j && cpu <= (uint32_t)(xj >> K10S_PK_SHIFT) && ram <= (xj & K10S_PK_RAM));
    }
    const uint32_t nf = (uint32_t)__popcll(front);
    const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(front >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)front, 0u));
    if (((front >> lane) & 1ull) && rank < K10S_FR_K) {
        fv[b * K10S_FR_K + rank] = x;
        fi[b * K10S_FR_K + rank] = (uint8_t)lane;
    }
    if (lane >= nf && lane < K10S_FR_K) fv[b * K10S_FR_K + lane] = 0;   // unused slots fit nothing
    return nf;
}
#endif
// Rebuild every marked block's front; returns the entries read.
K10S_HD_NOINL uint32_t fr_refresh(Ctx& c) {
    uint64_t dirty = uniform_u64(c.H().fr_dirty);
    if (dirty == 0) return 0;
    const uint32_t N = uniform_u32(c.S().n_nodes);
    const uint64_t* sn = c.V().s_node();
    uint64_t* fv = c.V().fr_val();
    uint8_t* fi = c.V().fr_idx();
    uint64_t over = uniform_u64(c.H().fr_over);
    uint32_t reads = 0;
#if K10S_DEVICE
    const uint32_t lane = (uint32_t)lane_id();
    while (dirty) {
        uint32_t bs[4];
        uint64_t xs[4];
        uint32_t k = 0;
        K10S_UNROLL
        for (uint32_t i = 0; i < 4; i++) {   // the next four marked blocks' loads together
            bs[i] = 0;
            xs[i] = 0;
            if (dirty) {
                const uint32_t b = (uint32_t)__builtin_ctzll(dirty);
                dirty &= dirty - 1;
                bs[i] = b;
                const uint32_t n = 64u * b + lane;
                if (n < N) xs[i] = sn[n];
                reads += N - 64u * b < 64u ? N - 64u * b : 64u;
                k = i + 1;
            }
        }
        K10S_UNROLL
        for (uint32_t i = 0; i < 4; i++) {
            if (i < k) {
                const uint32_t nf = fr_block(fv, fi, bs[i], xs[i]);
                over = nf > K10S_FR_K ? (over | (1ull << bs[i])) : (over & ~(1ull << bs[i]));
            }
        }
    }
#else
    while (dirty) {
        const uint32_t b = (uint32_t)__builtin_ctzll(dirty);
        dirty &= dirty - 1;
        const uint32_t lo = 64u * b, hi = lo + 64u < N ? lo + 64u : N;
        reads += hi - lo;
        uint32_t mem[64];
        uint32_t nf = 0;
        for (uint32_t k = hi; k-- > lo;) {   // from the last node: kept iff no kept later node dominates it
            const uint64_t x = sn[k];
            if (x == 0) continue;
            const NcEnt v = nc_unpack(x);
            bool dom = false;
            for (uint32_t q = 0; q < nf && !dom; q++) {
                const NcEnt w = nc_unpack(sn[mem[q]]);
                dom = w.cpu >= v.cpu && w.ram >= v.ram;
            }
            if (!dom) mem[nf++] = k;
        }
        for (uint32_t r = 0; r < K10S_FR_K; r++) {   // slots in ascending node order
            if (r < nf) {
                const uint32_t k = mem[nf - 1 - r];
                fv[b * K10S_FR_K + r] = sn[k];
                fi[b * K10S_FR_K + r] = (uint8_t)(k - lo);
            } else {
                fv[b * K10S_FR_K + r] = 0;
            }
        }
        over = nf > K10S_FR_K ? (over | (1ull << b)) : (over & ~(1ull << b));
    }
#endif
    c.H().fr_dirty = 0;
    c.H().fr_over = over;
    return reads;
}
// schedule_one over the fronts (fr_refresh first): K10S_SCHED_OK / NO_SUFFICIENT_RESOURCES;
// *nread: entries read.  Preconditions: weight 1.0, rc > 0, rr > 0, the cache packed with fronts.
K10S_HD_NOINL int front_scan(Ctx& c, uint32_t rc, uint64_t rr, int32_t* chosen, uint32_t* nread) {
    const uint32_t N = uniform_u32(c.S().n_nodes);
    const uint32_t NB = (N + 63u) >> 6;
    const uint64_t over = uniform_u64(c.H().fr_over);
    const uint64_t* fv = c.V().fr_val();
    const uint8_t* fi = c.V().fr_idx();
    const uint64_t* sn = c.V().s_node();
    uint32_t reads = NB * K10S_FR_K;
    uint64_t best_key = 0;
    int32_t best_n = -1;
#if K10S_DEVICE
    const uint32_t lane = (uint32_t)lane_id();
    rc = uniform_u32(rc);
    rr = uniform_u64(rr);
    const double frc = uniform_f64((double)rc), frr = uniform_f64(u64_f64(rr));
    const float fa = (float)rc;
    const float fr = __builtin_fmaf((float)(uint32_t)(rr >> 32), 4294967296.0f, (float)(uint32_t)rr);
    double bs = -__builtin_inf();
    int32_t bn = -1;
    uint64_t x[K10S_FR_K];
    uint64_t ix = 0;
    if (lane < NB) {
        const ulonglong2* p = reinterpret_cast<const ulonglong2*>(fv + lane * K10S_FR_K);
        K10S_UNROLL
        for (int k = 0; k < K10S_FR_K / 2; k++) {
            const ulonglong2 q = p[k];
            x[2 * k] = q.x;
            x[2 * k + 1] = q.y;
        }
        ix = *reinterpret_cast<const uint64_t*>(fi + lane * K10S_FR_K);
    } else {
        K10S_UNROLL
        for (int k = 0; k < K10S_FR_K; k++) x[k] = 0;
    }
    auto consider = [&](uint64_t e, int32_t n) {   // a fitting entry's exact score into the lane best
        const NcEnt v = nc_unpack(e);
        if (rc <= v.cpu && rr <= v.ram) {
            const double s = la_exact(v.cpu, v.ram, rr, frc, frr);
            if (s > bs || (s == bs && n > bn)) {
                bs = s;
                bn = n;
            }
        }
    };
    consider(x[0], (int32_t)(64u * lane + (uint32_t)(ix & 0xFFu)));
    float lu = bn >= 0 ? screen_u(bs) : __builtin_inff();
    const float thr = __builtin_bit_cast(float, uniform_u32(__builtin_bit_cast(uint32_t, wave_min_f32(lu))));
    const float T = thr + K10S_SCREEN_EPS;   // +inf when no lane scored: screens nothing out
#if K10S_FRONT_COMPACT
    // the screen of slots 1..7 first, then one exact scoring per round for each lane's next surviving
    // slot (rounds = the most survivors any lane has, not the slots any lane kept)
    uint32_t sm = 0;
    K10S_UNROLL
    for (int k = 1; k < K10S_FR_K; k++) {
        const NcEnt v = nc_unpack(x[k]);
        sm |= (x[k] != 0 && !scan_screen(v.cpu, v.ram, fa, fr, T)) ? 1u << k : 0u;
    }
    while (__ballot(sm != 0u)) {
        const uint32_t k = sm ? (uint32_t)__builtin_ctz(sm) : 0u;
        uint64_t e = x[1];
        K10S_UNROLL
        for (int q = 2; q < K10S_FR_K; q++) e = k == (uint32_t)q ? x[q] : e;
        if (sm) consider(e, (int32_t)(64u * lane + (uint32_t)((ix >> (8u * k)) & 0xFFu)));
        sm &= sm - 1u;
    }
#else
    K10S_UNROLL
    for (int k = 1; k < K10S_FR_K; k++) {
        const NcEnt v = nc_unpack(x[k]);
        if (x[k] != 0 && !scan_screen(v.cpu, v.ram, fa, fr, T))
            consider(x[k], (int32_t)(64u * lane + (uint32_t)((ix >> (8 * k)) & 0xFFu)));
    }
#endif
    // blocks whose front overflowed the slots (about 4 of 64 blocks per C3 scan): the whole block,
    // one node per lane, four blocks per memory round trip
    for (uint64_t ov = over; ov;) {
        uint32_t ob[4];
        uint64_t oe[4];
        K10S_UNROLL
        for (int i = 0; i < 4; i++) {
            ob[i] = 0xFFFFFFFFu;
            oe[i] = 0;
            if (ov) {
                const uint32_t b = (uint32_t)__builtin_ctzll(ov);
                ov &= ov - 1;
                ob[i] = 64u * b + lane;
                reads += N - 64u * b < 64u ? N - 64u * b : 64u;
                if (ob[i] < N) oe[i] = sn[ob[i]];
            }
        }
#if K10S_FRONT_COMPACT
        uint32_t om = 0;
        K10S_UNROLL
        for (int i = 0; i < 4; i++) {
            const NcEnt v = nc_unpack(oe[i]);
            om |= (oe[i] != 0 && !scan_screen(v.cpu, v.ram, fa, fr, T)) ? 1u << i : 0u;
        }
        while (__ballot(om != 0u)) {
            const uint32_t i = om ? (uint32_t)__builtin_ctz(om) : 0u;
            uint64_t e = oe[0];
            uint32_t n = ob[0];
            K10S_UNROLL
            for (int q = 1; q < 4; q++) {
                e = i == (uint32_t)q ? oe[q] : e;
                n = i == (uint32_t)q ? ob[q] : n;
            }
            if (om) consider(e, (int32_t)n);
            om &= om - 1u;
        }
#else
        K10S_UNROLL
        for (int i = 0; i < 4; i++) {
            const NcEnt v = nc_unpack(oe[i]);
            if (oe[i] != 0 && !scan_screen(v.cpu, v.ram, fa, fr, T)) consider(oe[i], (int32_t)ob[i]);
        }
#endif
    }
    best_key = bn >= 0 ? score_key(bs) : 0;
    best_n = bn;
    wave_argmax(best_key, best_n);
    best_n = (int32_t)uniform_u32((uint32_t)best_n);
#else
    for (uint32_t b = 0; b < NB; b++) {
        auto consider = [&](uint64_t e, int32_t n) {
            const NcEnt v = nc_unpack(e);
            if (e != 0 && rc <= v.cpu && rr <= v.ram) {
                const uint64_t k = score_key(la_score(v.cpu, v.ram, rc, rr));
                if (k > best_key || (k == best_key && n > best_n)) {
                    best_key = k;
                    best_n = n;
                }
            }
        };
        for (uint32_t k = 0; k < K10S_FR_K; k++) consider(fv[b * K10S_FR_K + k], (int32_t)(64u * b + fi[b * K10S_FR_K + k]));
        if ((over >> b) & 1ull) {
            const uint32_t hi = 64u * b + 64u < N ? 64u * b + 64u : N;
            reads += hi - 64u * b;
            for (uint32_t n = 64u * b; n < hi; n++) consider(sn[n], (int32_t)n);
        }
    }
#endif
    *nread = reads;
    if (best_n < 0) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    *chosen = best_n;
    return K10S_SCHED_OK;
}

// ---- score plugins beyond LeastAllocated alone (k10s_replica_params.score_plugins) --------------
// MostAllocatedResources is an extension: the reference registry (plugin.rs:13-23) has only Fit and
// LeastAllocatedResources.  Defined as kube-scheduler's MostAllocated strategy in this model's terms
// (requested = capacity − allocatable): per resource (capacity − allocatable + request)·100 /
// capacity, the two averaged like plugin.rs:52-63 averages its terms; u32 / u64 wrapping arithmetic
// (a fitting node has request <= allocatable <= capacity, so nothing wraps), 0/0 = NaN.
K10S_HD double ma_score(uint32_t ac, uint64_t ar, uint32_t cc, uint64_t cr, uint32_t rc, uint64_t rr) {
    double cpu_score = (double)(uint32_t)(cc - ac + rc) * 100.0 / (double)cc;
    double ram_score = (double)(uint64_t)(cr - ar + rr) * 100.0 / (double)cr;
    return (cpu_score + ram_score) / 2.0;
}
// The profile's weighted sum (kube_scheduler.rs:113-138): 0.0, then += score · weight per enabled
// plugin in registry order (LeastAllocated, MostAllocated).
K10S_HD double plugin_score(uint32_t ac, uint64_t ar, uint32_t cc, uint64_t cr, uint32_t rc, uint64_t rr,
                            uint32_t plugins, double w_la, double w_ma) {
    double s = 0.0;
    if (plugins & K10S_SCORE_LEAST_ALLOCATED) s += la_score(ac, ar, rc, rr) * w_la;
    if (plugins & K10S_SCORE_MOST_ALLOCATED) s += ma_score(ac, ar, cc, cr, rc, rr) * w_ma;
    return s;
}
// schedule_one with the plugin set (any weights, NaN and filtered[0] rules of kube_scheduler.rs:
// 140-148 as in schedule_scan): lanes stride the nodes (ascending per lane, "score >= best" keeps
// the lane's last maximum), then the cross-lane (score_key, index) max.  Reads the capacity SoA
// only for MostAllocated; IEEE divisions (the opt-in path is not the tuned one).
#ifndef K10S_SCORE_PLUGINS
#define K10S_SCORE_PLUGINS 1   // 0: the plugin path is not compiled (k10s_kernels.hip's default copy)
#endif
#if K10S_DEVICE
// plugin_score on the device, bit-identical: the same operations with la_score_d's division (rcp +
// Newton, exact for these integer operands with quotients in [0, 100]; 0/0 still gives NaN) and
// (c + r) / 2.0 as an exact halving.
K10S_D double ma_score_d(uint32_t ac, uint64_t ar, uint32_t cc, uint64_t cr, uint32_t rc, uint64_t rr) {
    const double cs = div_rn((double)(uint32_t)(cc - ac + rc) * 100.0, (double)cc);
    const double rs = div_rn(u64_f64((uint64_t)(cr - ar + rr)) * 100.0, u64_f64(cr));
    return (cs + rs) * 0.5;
}
K10S_D double plugin_score_d(uint32_t ac, uint64_t ar, uint32_t cc, uint64_t cr, uint32_t rc, uint64_t rr,
                             uint32_t plugins, double w_la, double w_ma) {
    double s = 0.0;
    if (plugins & K10S_SCORE_LEAST_ALLOCATED) s += la_score_d(ac, ar, rc, rr) * w_la;
    if (plugins & K10S_SCORE_MOST_ALLOCATED) s += ma_score_d(ac, ar, cc, cr, rc, rr) * w_ma;
    return s;
}
K10S_D void plugin_node(uint32_t n, bool present, uint32_t ac, uint64_t ar, uint32_t cc, uint64_t cr, uint32_t rc,
                        uint64_t rr, uint32_t plugins, double w_la, double w_ma, int32_t& first, uint64_t& best_key,
                        int32_t& best_n) {
    if (present && rc <= ac && rr <= ar) {
        first = (int32_t)n < first ? (int32_t)n : first;
        const double s = plugin_score_d(ac, ar, cc, cr, rc, rr, plugins, w_la, w_ma);
        if (!is_nan(s)) {
            const uint64_t k = score_key(s);
            if (k >= best_key) {
                best_key = k;
                best_n = (int32_t)n;
            }
        }
    }
}
#endif
K10S_HD int schedule_scan_plugins(Ctx& c, uint32_t rc, uint64_t rr, int32_t* chosen) {
    const uint32_t N = c.S().n_nodes;
    const uint32_t* cpu = c.V().s_cpu();
    const uint64_t* ram = c.V().s_ram();
    const uint32_t* ccpu = c.V().s_ccpu();
    const uint64_t* cram = c.V().s_cram();
    const uint64_t* pres = c.V().s_present();
    const uint32_t plugins = c.P().score_plugins;
    const double w_la = c.P().score_weight, w_ma = c.P().most_allocated_weight;
    uint64_t best_key = 0;
    int32_t best_n = -1;
    int32_t first = 0x7fffffff;
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_SCAN_PLUGINS)) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    // each lane owns 4 consecutive nodes per 256-node step, as the LeastAllocated scan: one 16-B
    // load per u32 array and two per u64 array (sections 256-B aligned and padded; a lane past the
    // end re-reads nodes 0..3 and grp_bits masks them out); ascending per lane, then the cross-lane
    // (score_key, index) max reproduces the left-to-right argmax
    rc = uniform_u32(rc);
    rr = uniform_u64(rr);
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    for (uint32_t base = 0; base < N; base += 256) {
        const uint32_t n0 = base + l4;
        const ScanGrp g = scan_load(cpu, ram, pres, N, n0);
        const uint32_t a = n0 < N ? n0 : 0u;
        const uint4 cc = *reinterpret_cast<const uint4*>(ccpu + a);
        const ulonglong2 c01 = *reinterpret_cast<const ulonglong2*>(cram + a);
        const ulonglong2 c23 = *reinterpret_cast<const ulonglong2*>(cram + a + 2);
        const uint32_t bits = grp_bits(g, n0, N);
        if (bits) {
            plugin_node(n0, bits & 1u, g.cv.x, g.r01.x, cc.x, c01.x, rc, rr, plugins, w_la, w_ma, first, best_key, best_n);
            plugin_node(n0 + 1, bits & 2u, g.cv.y, g.r01.y, cc.y, c01.y, rc, rr, plugins, w_la, w_ma, first, best_key, best_n);
            plugin_node(n0 + 2, bits & 4u, g.cv.z, g.r23.x, cc.z, c23.x, rc, rr, plugins, w_la, w_ma, first, best_key, best_n);
            plugin_node(n0 + 3, bits & 8u, g.cv.w, g.r23.y, cc.w, c23.y, rc, rr, plugins, w_la, w_ma, first, best_key, best_n);
        }
    }
    first = wave_min_i32(first);
    wave_argmax(best_key, best_n);
    if (first == 0x7fffffff) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    const uint32_t f = (uint32_t)uniform_u32((uint32_t)first);
    const double s0 = plugin_score_d(cpu[f], ram[f], ccpu[f], cram[f], rc, rr, plugins, w_la, w_ma);
    *chosen = is_nan(s0) ? (int32_t)f : best_n;
    return K10S_SCHED_OK;
#else
    for (uint32_t n = (uint32_t)lane_id(); n < N; n += K10S_LANES) {
        if (!bit_test(pres, n)) continue;
        const uint32_t ac = cpu[n];
        const uint64_t ar = ram[n];
        if (rc <= ac && rr <= ar) {
            if ((int32_t)n < first) first = (int32_t)n;
            const double s = plugin_score(ac, ar, ccpu[n], cram[n], rc, rr, plugins, w_la, w_ma);
            if (!is_nan(s)) {
                const uint64_t k = score_key(s);
                if (k >= best_key) {
                    best_key = k;
                    best_n = (int32_t)n;
                }
            }
        }
    }
    first = wave_min_i32(first);
    wave_argmax(best_key, best_n);
    if (first == 0x7fffffff) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    const uint32_t f = (uint32_t)uniform_u32((uint32_t)first);
    const double s0 = plugin_score(cpu[f], ram[f], ccpu[f], cram[f], rc, rr, plugins, w_la, w_ma);
    *chosen = is_nan(s0) ? (int32_t)f : best_n;
    return K10S_SCHED_OK;
#endif
}

// ---- block bounds of the scheduler cache and the exact pruned scan ------------------------------
// The node cache is cut into blocks of 2^bshift consecutive indices (64 <= block, <= 64 blocks);
// s_bcpu[b] / s_bram[b] hold the largest allocatable cpu / ram over the block's present nodes (0 if
// none), recomputed whenever a node of the block changes (reserve, release, add, remove).
//
// Why a bound is exact: with rc > 0, rr > 0 and every ram below 2^46, each LeastAllocated term is
// a correctly rounded quotient of exactly represented integers (100·(a − r) < 2^53, a < 2^53) whose
// real value 100·(1 − r/a) grows with a, and rounding is monotone, so the f64 score
// ((c + r) / 2.0, weight 1.0) of any fitting node is <= the f64 score of (bcpu[b], bram[b]).  A
// block whose bound is below the best exact score found so far — or equal to it with all its
// indices below the best node (ties go to the last node in name order, kube_scheduler.rs:140-148)
// — cannot contain the argmax; rc, rr > 0 also rules out the 0/0 NaN of filtered[0].
K10S_HD void block_recompute(Ctx& c, uint32_t b) {
    const uint32_t N = c.S().n_nodes, sh = c.Ly().bshift;
    const uint32_t lo = b << sh;
    const uint32_t hi = (lo + (1u << sh)) < N ? (lo + (1u << sh)) : N;
    const uint32_t* cpu = c.V().s_cpu();
    const uint64_t* ram = c.V().s_ram();
    const uint64_t* pres = c.V().s_present();
    uint32_t mc = 0;
    uint64_t mr = 0;
    for (uint32_t n = lo + (uint32_t)lane_id(); n < hi; n += K10S_LANES) {
        if ((pres[n >> 6] >> (n & 63)) & 1ull) {
            uint32_t x = cpu[n];
            uint64_t y = ram[n];
            mc = x > mc ? x : mc;
            mr = y > mr ? y : mr;
        }
    }
    mc = wave_max_u32(mc);
    mr = wave_max_u64(mr);
    c.V().s_bcpu()[b] = mc;
    c.V().s_bram()[b] = mr;
    c.H().counters[K10S_C_NODES_READ] += hi - lo;
}
K10S_HD void node_bound_changed(Ctx& c, uint32_t n) {
    if (nc_packed(c) || !c.Ly().pruned) return;   // bounds: pruned scans only, wide layout only
    const uint64_t t0 = prof_now();
    block_recompute(c, n >> c.Ly().bshift);
    K10S_PROF_ADD(c, PROF_BOUNDS, t0);
}

// Returns K10S_SCHED_OK / NO_SUFFICIENT_RESOURCES, or -1 when the bound argument does not apply
// (a block maximum of ram >= 2^46): the caller then runs the full scan.  Preconditions (caller):
// weight == 1.0, rc > 0, rr > 0.  *nread = scheduler-cache entries read (bounds + scanned blocks).
K10S_HD int schedule_scan_pruned(Ctx& c, uint32_t rc, uint64_t rr, int32_t* chosen, uint32_t* nread) {
    const uint32_t N = c.S().n_nodes, NB = c.Ly().nblocks, sh = c.Ly().bshift;
    const uint32_t* bc = c.V().s_bcpu();
    const uint64_t* br = c.V().s_bram();
    const uint32_t* cpu = c.V().s_cpu();
    const uint64_t* ram = c.V().s_ram();
    const uint64_t* pres = c.V().s_present();
    const uint64_t BIG = 1ull << 46;
    uint32_t touched = NB;
    uint64_t best_key = 0;
    int32_t best_n = -1;
#if K10S_DEVICE
    // lane b holds block b's bound key (0: no node of the block can fit)
    const uint32_t lane = (uint32_t)lane_id();
    uint64_t bkey = 0;
    bool big = false;
    if (lane < NB) {
        const uint32_t A = bc[lane];
        const uint64_t Rm = br[lane];
        big = Rm >= BIG;
        if (A >= rc && Rm >= rr) bkey = score_key(la_score(A, Rm, rc, rr));
    }
    if (wave_any(big)) return -1;
    for (;;) {
        uint64_t k = bkey;
        int32_t bi = bkey ? (int32_t)lane : -1;
        wave_argmax(k, bi);
        // every lane holds the reduced pair; saying so keeps this loop's branches scalar (a divergent
        // structurization would run the next wave_argmax under a partial EXEC: tools/divergent_loops.py)
        k = uniform_u64(k);
        bi = (int32_t)uniform_u32((uint32_t)bi);
        if (k == 0) break;
        if (best_n >= 0 && (k < best_key || (k == best_key && (int32_t)(((uint32_t)bi + 1u) << sh) <= best_n))) break;
        const uint32_t lo = (uint32_t)bi << sh;
        const uint32_t hi = (lo + (1u << sh)) < N ? (lo + (1u << sh)) : N;
        uint64_t lk = 0;
        int32_t ln = -1;
        for (uint32_t n = lo + lane; n < hi; n += 64) {
            if ((pres[n >> 6] >> (n & 63)) & 1ull) {
                const uint32_t ac = cpu[n];
                const uint64_t ar = ram[n];
                if (rc <= ac && rr <= ar) {
                    const uint64_t kk = score_key(la_score(ac, ar, rc, rr));
                    if (kk >= lk) {
                        lk = kk;
                        ln = (int32_t)n;
                    }
                }
            }
        }
        touched += hi - lo;
        wave_argmax(lk, ln);
        lk = uniform_u64(lk);
        ln = (int32_t)uniform_u32((uint32_t)ln);
        if (ln >= 0 && (lk > best_key || (lk == best_key && ln > best_n))) {
            best_key = lk;
            best_n = ln;
        }
        if ((int32_t)lane == bi) bkey = 0;
    }
#else
    uint64_t keys[64];
    for (uint32_t b = 0; b < NB; b++) {
        if (br[b] >= BIG) return -1;
        keys[b] = (bc[b] >= rc && br[b] >= rr) ? score_key(la_score(bc[b], br[b], rc, rr)) : 0;
    }
    for (;;) {
        uint64_t k = 0;
        int32_t bi = -1;
        for (uint32_t b = 0; b < NB; b++)
            if (keys[b] && keys[b] >= k) {
                k = keys[b];
                bi = (int32_t)b;
            }
        if (k == 0) break;
        if (best_n >= 0 && (k < best_key || (k == best_key && (int32_t)(((uint32_t)bi + 1u) << sh) <= best_n))) break;
        const uint32_t lo = (uint32_t)bi << sh;
        const uint32_t hi = (lo + (1u << sh)) < N ? (lo + (1u << sh)) : N;
        for (uint32_t n = lo; n < hi; n++) {
            if (!((pres[n >> 6] >> (n & 63)) & 1ull)) continue;
            if (rc <= cpu[n] && rr <= ram[n]) {
                const uint64_t kk = score_key(la_score(cpu[n], ram[n], rc, rr));
                if (kk > best_key || (kk == best_key && (int32_t)n > best_n)) {  // (key, index) max
                    best_key = kk;
                    best_n = (int32_t)n;
                }
            }
        }
        touched += hi - lo;
        keys[bi] = 0;
    }
#endif
    *nread = touched;
    if (best_n < 0) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    *chosen = best_n;
    return K10S_SCHED_OK;
}

// ---- batched fit pass of a cycle tile (exact early fail) -----------------------------------------
// Nothing is pushed onto the action queue during a cycle (scheduler.rs:261-330: a failed pod goes to
// the unschedulable map, every emission to the event queue), so the cycle's pod sequence is fixed
// when it starts, and the only change the cycle makes to the node cache is reserve_node_resources
// (scheduler.rs:118-123), which lowers one node's allocatable.  So a pod that fits no node of the
// cache as it is when its tile is formed fits no node when its turn comes: its attempt fails with
// NoSufficientResources (kube_scheduler.rs:89-97), exactly as the scan would find.  The fit pass
// answers "fits some node?" for K10S_TILE pods with one read of the node cache (packed entries, two
// 16-B loads per lane per 512 nodes as the screened scan; per node and pod one 32-bit and one 64-bit
// compare into lane masks), and stops as soon as every pod of the tile has a fitting node.  Pods
// that fit are then scheduled one at a time by the exact scan, in order, on the current cache.
// Used only after a cycle with failed attempts (RepHdr::cyc_fails): in the light regime every pod
// fits and the pass would only add reads; in the backlog regime most attempts fail and their node
// scans become one shared read per tile.
#ifndef K10S_TILE
#define K10S_TILE 32   // round 5: 8 -> 32, backlog -3 % and 6,511 -> 5,032 entries read per placement (r05_ab18)
#endif
static_assert(K10S_TILE >= 1 && K10S_TILE <= 32, "K10S_TILE");
// Bit j set: pod j of the tile (need bit j: request rc8[j] = cpu << 8, rr[j] = ram, both > 0 and cpu
// < 2^24) fits some node of the packed cache (cpu field >= cpu, ram field >= ram).  Absent nodes hold
// (0, 0) and fit nothing.  *nread: cache entries read.
// bnd (not NULL, block size 2^sh with 6 <= sh <= 8): the pass reads the whole cache and leaves each
// block's bound in bnd[b] (tile_scan_pruned below).
#if K10S_DEVICE
template <int S>
K10S_D void bmax_step(uint32_t& c, uint64_t& r) {
    uint32_t a, b, la, lb, ha, hb;
    xpair<S>(c, a, b);
    c = a > b ? a : b;
    xpair<S>((uint32_t)r, la, lb);
    xpair<S>((uint32_t)(r >> 32), ha, hb);
    const uint64_t ra = join64(la, ha), rb = join64(lb, hb);
    r = ra > rb ? ra : rb;
}
// (cpu, ram) maxima over the 2^(sh-2) lanes of a block (every lane of the group gets them)
K10S_D void block_max(uint32_t& c, uint64_t& r, uint32_t sh) {
    bmax_step<0>(c, r);
    bmax_step<1>(c, r);
    bmax_step<2>(c, r);
    bmax_step<3>(c, r);
    if (sh >= 7) bmax_step<4>(c, r);
    if (sh >= 8) bmax_step<5>(c, r);
}
#endif
K10S_HD uint32_t fit_tile(const uint64_t* s_node, uint32_t n_nodes, const uint32_t* rc8, const uint64_t* rr,
                          uint32_t need, uint32_t* nread, uint64_t* bnd = nullptr, uint32_t sh = 6) {
    uint32_t found = 0;
#if K10S_DEVICE
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    const bool wb = bnd != nullptr;   // wave-uniform
    uint32_t base = 0;
    for (; base < n_nodes && (wb || (found & need) != need); base += 512) {
        // a lane's 8 nodes of this 512-node block (past the end: entries 0..3 re-read, then zeroed)
        const uint32_t a0 = base + l4, a1 = base + 256u + l4;
        const uint32_t b0 = a0 < n_nodes ? a0 : 0u, b1 = a1 < n_nodes ? a1 : 0u;
        const ulonglong2 p0 = *reinterpret_cast<const ulonglong2*>(s_node + b0);
        const ulonglong2 p1 = *reinterpret_cast<const ulonglong2*>(s_node + b0 + 2);
        const ulonglong2 p2 = *reinterpret_cast<const ulonglong2*>(s_node + b1);
        const ulonglong2 p3 = *reinterpret_cast<const ulonglong2*>(s_node + b1 + 2);
        uint64_t x[8] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};
        if (base + 512u > n_nodes) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t n = (k < 4 ? a0 : a1) + (uint32_t)(k & 3);
                x[k] = n < n_nodes ? x[k] : 0ull;
            }
        }
        uint32_t hi[8];
        uint64_t ram[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            hi[k] = (uint32_t)(x[k] >> 32);      // cpu << 8 | ram >> 32
            ram[k] = x[k] & K10S_PK_RAM;
        }
#pragma unroll
        for (int j = 0; j < K10S_TILE; j++) {
            if (!((need & ~found) >> j & 1u)) continue;   // wave-uniform
            bool f = false;
#pragma unroll
            for (int k = 0; k < 8; k++) f |= hi[k] >= rc8[j] && ram[k] >= rr[j];
            if (__ballot(f)) found |= 1u << j;
        }
        if (wb) {   // the blocks' (cpu, ram) maxima: lane-local over 4 entries, then over the block's lanes
            uint32_t ca = 0, cb = 0;
            uint64_t ra = 0, rb = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                ca = (hi[k] >> 8) > ca ? (hi[k] >> 8) : ca;
                ra = ram[k] > ra ? ram[k] : ra;
                cb = (hi[k + 4] >> 8) > cb ? (hi[k + 4] >> 8) : cb;
                rb = ram[k + 4] > rb ? ram[k + 4] : rb;
            }
            block_max(ca, ra, sh);
            block_max(cb, rb, sh);
            if ((l4 & ((4u << (sh - 2)) - 1u)) == 0) {   // the block's first lane writes its bound
                if (a0 < n_nodes) bnd[a0 >> sh] = nc_pack(ca, ra);
                if (a1 < n_nodes) bnd[a1 >> sh] = nc_pack(cb, rb);
            }
        }
    }
    *nread = base < n_nodes ? base : n_nodes;
#else
    uint32_t n = 0;
    if (bnd)
        for (uint32_t b = 0; (b << sh) < n_nodes; b++) bnd[b] = 0;
    for (; n < n_nodes && (bnd || (found & need) != need); n++) {
        const uint64_t x = s_node[n];
        for (int j = 0; j < K10S_TILE; j++)
            if ((need >> j & 1u) && (uint32_t)(x >> 32) >= rc8[j] && (x & K10S_PK_RAM) >= rr[j]) found |= 1u << j;
        if (bnd) {
            const NcEnt v = nc_unpack(x), b = nc_unpack(bnd[n >> sh]);
            bnd[n >> sh] = nc_pack(v.cpu > b.cpu ? v.cpu : b.cpu, v.ram > b.ram ? v.ram : b.ram);
        }
    }
    *nread = n;
#endif
    return found;
}

// ---- pruned scans inside a cycle tile (round 6) ---------------------------------------------------
// The tile's fit pass (fit_tile with bnd) reads the whole packed cache and leaves, per block of 2^sh
// consecutive nodes (the layout's nblocks <= 64 blocks, 6 <= sh <= 8), the componentwise maximum
// (cpu, ram) of the block's entries.  Until the tile ends the cycle changes the cache only by
// reserve_node_resources (scheduler.rs:118-123), which lowers an entry, so each bound stays >= every
// entry of its block.  A fitting pod of the tile then scans blocks best bound first and stops when
// no unvisited block can hold the argmax: with rc, rr > 0 (no 0/0), the LeastAllocated score is
// monotone in (cpu, ram) (schedule_scan_pruned's argument: correctly rounded quotients of exactly
// represented integers), so a node's score is <= its block bound's, and a block whose bound score is
// below the best found — or equal with every index below the best node (the last maximum in name
// order wins, kube_scheduler.rs:140-148) — is skipped.  A bound that fits no request means no node of
// the block fits.  Measured on the host (tools/prune_study.py, 64-node blocks with tight bounds): the
// backlog's fitting pods visit 1.02 blocks per scan (129 of 4,096 entries); C3's light regime 47
// blocks (74 %), which is why the serial cycle (C3) keeps the screened full scan.  More than
// K10S_TILE_PRUNE_MAX visited blocks fall back to the full scan (same result).  A visited block's bound
// is tightened to its entries' maxima (the scan reads them all), so a block that an earlier pod of
// the tile reserved on is not left looking better than it is.
// Measured and not kept (default 0, profiles/r06_g1_tile_prune_ab.json, r06_g2_aq_sorted_ab.json): the
// backlog line reads 2,660 instead of 5,032 node-cache entries per placement, but its time does not
// fall (1,990 -> 1,989-1,997 ms; with the sorted action queue 1,804 -> 1,844-1,857 ms) — those scans
// are not on the backlog's critical path — and the larger tile function moves the run kernel's
// register allocation (C3 -0.5 to +1 %).  Kept as a knob with its parity tests (tests/test_cycle_tile.py).
#ifndef K10S_TILE_PRUNE
#define K10S_TILE_PRUNE 0
#endif
#ifndef K10S_TILE_PRUNE_MAX
#define K10S_TILE_PRUNE_MAX 6
#endif
// Returns K10S_SCHED_OK / NO_SUFFICIENT_RESOURCES, or -1 (fall back to the full scan).  *nread:
// entries read (bounds + visited blocks).  Preconditions: weight 1.0, rc > 0, rr > 0, both within
// the packed fields.
K10S_HD_NOINL int tile_scan_pruned(const uint64_t* s_node, uint64_t* bnd, uint32_t N, uint32_t sh, uint32_t rc,
                             uint64_t rr, int32_t* chosen, uint32_t* nread) {
    const uint32_t NB = (N + (1u << sh) - 1u) >> sh;
    uint32_t reads = NB, visits = 0;
    uint64_t best_key = 0;
    int32_t best_n = -1;
#if K10S_DEVICE
    const uint32_t lane = (uint32_t)lane_id();
    rc = uniform_u32(rc);
    rr = uniform_u64(rr);
    const double frc = uniform_f64((double)rc), frr = uniform_f64(u64_f64(rr));
    uint64_t bkey = 0;   // lane b: block b's bound score key (0: nothing in the block fits)
    if (lane < NB) {
        const NcEnt v = nc_unpack(bnd[lane]);
        if (rc <= v.cpu && rr <= v.ram) bkey = score_key(la_exact(v.cpu, v.ram, rr, frc, frr));
    }
    for (;;) {
        const int32_t last = (int32_t)(((lane + 1u) << sh) - 1u);   // block's largest index
        const bool alive = bkey != 0 && (best_n < 0 || bkey > best_key || (bkey == best_key && last > best_n));
        uint64_t k = alive ? bkey : 0;
        int32_t bi = alive ? (int32_t)lane : -1;
        wave_argmax(k, bi);
        bi = (int32_t)uniform_u32((uint32_t)bi);
        if (bi < 0) break;
        if (visits == K10S_TILE_PRUNE_MAX) {
            *nread = reads;
            return -1;
        }
        visits++;
        const uint32_t lo = (uint32_t)bi << sh, hi = (lo + (1u << sh)) < N ? (lo + (1u << sh)) : N;
        uint64_t lk = 0;
        int32_t ln = -1;
        uint32_t mc = 0;   // the block's (cpu, ram) maxima: its bound, tightened (reservations earlier in
        uint64_t mr = 0;   // the tile left it above the entries)
        for (uint32_t m = lo; m < hi; m += 64) {   // lane i: nodes lo + i, lo + 64 + i, ... (ascending)
            const uint32_t n = m + lane;
            if (n < hi) {
                const NcEnt v = nc_unpack(s_node[n]);
                mc = v.cpu > mc ? v.cpu : mc;
                mr = v.ram > mr ? v.ram : mr;
                if (rc <= v.cpu && rr <= v.ram) {
                    const uint64_t kk = score_key(la_exact(v.cpu, v.ram, rr, frc, frr));
                    if (kk >= lk) {
                        lk = kk;
                        ln = (int32_t)n;
                    }
                }
            }
        }
        reads += hi - lo;
        block_max(mc, mr, 8);
        if (lane == 0) bnd[bi] = nc_pack(mc, mr);
        wave_argmax(lk, ln);
        lk = uniform_u64(lk);
        ln = (int32_t)uniform_u32((uint32_t)ln);
        if (ln >= 0 && (lk > best_key || (lk == best_key && ln > best_n))) {
            best_key = lk;
            best_n = ln;
        }
        if (lane == (uint32_t)bi) bkey = 0;
    }
#else
    uint64_t keys[64];
    for (uint32_t b = 0; b < NB; b++) {
        const NcEnt v = nc_unpack(bnd[b]);
        keys[b] = (rc <= v.cpu && rr <= v.ram) ? score_key(la_score(v.cpu, v.ram, rc, rr)) : 0;
    }
    for (;;) {
        int32_t bi = -1;
        uint64_t k = 0;
        for (uint32_t b = 0; b < NB; b++) {
            const int32_t last = (int32_t)(((b + 1u) << sh) - 1u);
            const bool alive = keys[b] != 0 && (best_n < 0 || keys[b] > best_key || (keys[b] == best_key && last > best_n));
            if (alive && keys[b] >= k) {   // (key, block) maximum: the device's wave_argmax
                k = keys[b];
                bi = (int32_t)b;
            }
        }
        if (bi < 0) break;
        if (visits == K10S_TILE_PRUNE_MAX) {
            *nread = reads;
            return -1;
        }
        visits++;
        const uint32_t lo = (uint32_t)bi << sh, hi = (lo + (1u << sh)) < N ? (lo + (1u << sh)) : N;
        uint32_t mc = 0;
        uint64_t mr = 0;
        for (uint32_t n = lo; n < hi; n++) {
            const NcEnt v = nc_unpack(s_node[n]);
            mc = v.cpu > mc ? v.cpu : mc;
            mr = v.ram > mr ? v.ram : mr;
            if (rc <= v.cpu && rr <= v.ram) {
                const uint64_t kk = score_key(la_score(v.cpu, v.ram, rc, rr));
                if (kk > best_key || (kk == best_key && (int32_t)n > best_n)) {
                    best_key = kk;
                    best_n = (int32_t)n;
                }
            }
        }
        reads += hi - lo;
        bnd[bi] = nc_pack(mc, mr);
        keys[bi] = 0;
    }
#endif
    *nread = reads;
    if (best_n < 0) return K10S_SCHED_NO_SUFFICIENT_RESOURCES;
    *chosen = best_n;
    return K10S_SCHED_OK;
}

// ---- best-node pass of a cycle tile (exact picks for the pods that fit) --------------------------
// K10S_TILE_BEST=1: the tile's shared read also finds where each pod of the tile goes, and the pods
// that fit are placed from it instead of by one full scan each.
// Lanes: node n belongs to lane (n >> 2) & 63, the scans' layout (a lane's 4 consecutive nodes of
// every 256-node step); S_L is lane L's share.  For every pod j of the tile and every lane L the pass
// keeps b_jL, the (score, index) maximum over the nodes of S_L that fit j in the cache as it is when
// the tile is formed (the snapshot).  Its screen (scan_screen) compares a node only with nodes the
// same lane scored before, so b_jL is exactly that maximum.
// Why the picks are the reference's: between the snapshot and pod j's turn the cycle changes the
// cache only by reserve_node_resources on the nodes R that earlier pods of the tile were assigned
// (scheduler.rs:118-123; nothing else runs inside a cycle, fit_tile above), so every node outside R
// still has its snapshot entry.  The reference picks the (score, index) maximum over the nodes that
// fit now (kube_scheduler.rs:140-148 over the name-ordered nodes, the last maximum), which is the
// maximum over lanes of the maximum over S_L.  A lane whose share holds no node of R has all of its
// nodes unchanged, so its maximum is b_jL.  Every other lane (at most |R| <= K10S_TILE - 1 of them)
// rescans its own share under the current cache: n_nodes/64 entries per flagged lane, all flagged
// lanes together.  The maximum of the lane values is the pick, and no lane value means no node fits
// (NoSufficientResources).  A pod that fits no node of the snapshot fits none now (fit_tile above).
// The pass costs one read of the cache per tile; a placement otherwise costs a full read of its own.
// Measured and not kept (default 0, profiles/r05_ab5_windows_tile_best.json): on the backlog line it cuts
// the entries read per placement from 6,511 to 4,467 but takes 3,780 ms per launch instead of 2,290
// (the pass's per-pod lane state spills at 64 VGPRs, 74 % of the picks need a rescan, and the
// cycle's bookkeeping, not its reads, dominates that regime); C3 never runs tiles but lost 2.7 % to
// the larger callee's register clobbers.  Kept as a knob with its parity tests
// (tests/test_cycle_tile.py::test_tile_best_variant_host).
#ifndef K10S_TILE_BEST
#define K10S_TILE_BEST 0
#endif
// Tile pod j's request: rc, rr (> 0, within the packed fields), their f64 and f32 forms.
struct TileReq {
    K10S_GB(const PodState) P;   // the pod's line: the exact test reads the requests from it
    float fa, fr;                // device: the request as f32 (the screen)
};
K10S_HD TileReq tile_req(K10S_GB(const PodState) P, uint32_t rc, uint64_t rr) {
    TileReq q;
#if K10S_DEVICE
    // all wave-uniform: kept in SGPRs through the pass
    q.P = P;
    q.fa = __builtin_bit_cast(float, uniform_u32(__builtin_bit_cast(uint32_t, (float)rc)));
    q.fr = __builtin_bit_cast(float, uniform_u32(__builtin_bit_cast(uint32_t, __builtin_fmaf((float)(uint32_t)(rr >> 32), 4294967296.0f, (float)(uint32_t)rr))));
#else
    q.P = P;
    q.fa = q.fr = 0.0f;
#endif
    return q;
}
#if K10S_DEVICE
// A lane's 4 consecutive packed entries at n0 (clamped address, as scan_load_pk) and, once for all
// pods of the tile, their allocatables as f32 (the screen's A and R).  The f32 conversions are
// monotone (R = fl(hi·2^32 + fl(lo)) rounds twice, both monotone; the request's fa, fr the same
// way), so a node that fits (cpu >= rc, ram >= rr) has A >= fa and R >= fr: the f32 test keeps every
// fitting node, and the survivors are tested exactly on the entry, reloaded.
struct TileGrp {
    f32x2 A01, A23, R01, R23;
};
typedef K10S_GB(const uint64_t) NodeCachePtr;   // the packed cache, global address space
K10S_D void tile_load(ulonglong2 (&x)[2], NodeCachePtr s_node, uint32_t n_nodes, uint32_t n0) {
    const uint32_t a = n0 < n_nodes ? n0 : 0u;
    x[0] = *reinterpret_cast<K10S_GB(const ulonglong2)>(s_node + a);
    x[1] = *reinterpret_cast<K10S_GB(const ulonglong2)>(s_node + a + 2);
}
K10S_D TileGrp tile_convert(const ulonglong2 (&x)[2]) {
    const uint64_t e[4] = {x[0].x, x[0].y, x[1].x, x[1].y};
    float A[4], R[4];
    K10S_UNROLL
    for (int k = 0; k < 4; k++) {
        const uint32_t hi = (uint32_t)(e[k] >> 32);
        A[k] = cvt_f32_u32(hi >> 8);
        R[k] = __builtin_fmaf(cvt_f32_u32(hi & 0xFFu), 4294967296.0f, cvt_f32_u32((uint32_t)e[k]));
    }
    TileGrp g;
    g.A01 = f32x2{A[0], A[1]};
    g.A23 = f32x2{A[2], A[3]};
    g.R01 = f32x2{R[0], R[1]};
    g.R23 = f32x2{R[2], R[3]};
    return g;
}
// One pod over a lane's group at n0 (bits: the nodes in range): the f32 fit test, the screen against
// the lane's own best (scan_screen; T from its score, +inf before it has one), then the survivors in
// ascending order: exact Fit on the reloaded entry (absent nodes hold 0 and fit nothing), the exact
// score, ">=" keeping the last maximum.
K10S_D void tile_best_grp(const TileGrp& g, uint32_t bits, NodeCachePtr s_node, uint32_t n0, const TileReq& q,
                          double& bs, int32_t& bn) {
    const float T = bn < 0 ? __builtin_inff() : screen_u(bs) + K10S_SCREEN_EPS;
    const f32x2 va = {q.fa, q.fa}, vr = {q.fr, q.fr}, vT = {T, T};
    const f32x2 l01 = __builtin_elementwise_fma(va, g.R01, vr * g.A01), l23 = __builtin_elementwise_fma(va, g.R23, vr * g.A23);
    const f32x2 r01 = (g.A01 * g.R01) * vT, r23 = (g.A23 * g.R23) * vT;
    const uint32_t keep = (uint32_t)(g.A01.x >= q.fa && g.R01.x >= q.fr && !(l01.x > r01.x)) |
                          ((uint32_t)(g.A01.y >= q.fa && g.R01.y >= q.fr && !(l01.y > r01.y)) << 1) |
                          ((uint32_t)(g.A23.x >= q.fa && g.R23.x >= q.fr && !(l23.x > r23.x)) << 2) |
                          ((uint32_t)(g.A23.y >= q.fa && g.R23.y >= q.fr && !(l23.y > r23.y)) << 3);
    uint32_t need = keep & bits;
    // one exact test in the code (an innermost loop, no calls)
    while (need) {
        const uint32_t k = (uint32_t)__builtin_ctz(need);
        need &= need - 1u;
        const uint64_t x = s_node[n0 + k];
        const uint32_t ac = (uint32_t)(x >> K10S_PK_SHIFT);
        const uint64_t ar = x & K10S_PK_RAM;
        const uint32_t rc = uniform_u32(q.P->req_cpu);
        const uint64_t rr = uniform_u64(q.P->req_ram);
        if (rc <= ac && rr <= ar) {
            const double s = la_exact(ac, ar, rr, (double)rc, u64_f64(rr));
            if (s >= bs) {
                bs = s;
                bn = (int32_t)(n0 + k);
            }
        }
    }
}
K10S_D uint32_t tile_bits(uint32_t n0, uint32_t n_nodes) {
    return n0 < n_nodes ? (n_nodes - n0 >= 4 ? 0xFu : (1u << (n_nodes - n0)) - 1u) : 0u;
}
// The pass: b_jL for every pod j of need (bs: score, bn: index, -1 none), one read of the cache,
// one 256-node step per iteration with the next step's loads in flight.  Out of line (its own
// registers: 8 pods' lane state, 24 VGPRs, beside the cycle's); the tile's pod j is the queue entry
// at slot_top[sdir * j], its requests read here.
__device__ __attribute__((noinline)) void tile_best_pass(NodeCachePtr s_node, uint32_t n_nodes,
                                                        K10S_GB(const QInfo) slot_top, int32_t sdir,
                                                        K10S_GB(const PodState) pods, uint32_t need, double* bs,
                                                        int32_t* bn) {
    // (a callee's arguments arrive in VGPRs: say which are wave-uniform)
    s_node = (NodeCachePtr)uniform_u64((uint64_t)s_node);
    slot_top = (K10S_GB(const QInfo))uniform_u64((uint64_t)slot_top);
    sdir = (int32_t)uniform_u32((uint32_t)sdir);
    pods = (K10S_GB(const PodState))uniform_u64((uint64_t)pods);
    n_nodes = uniform_u32(n_nodes);
    need = uniform_u32(need);
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    TileReq q[K10S_TILE];
    K10S_UNROLL
    for (int j = 0; j < K10S_TILE; j++) {
        if ((need >> j) & 1u) {
            const uint32_t p = uniform_u32(slot_top[sdir * j].pod);
            q[j] = tile_req(pods + p, pods[p].req_cpu, pods[p].req_ram);
        } else {
            q[j] = tile_req(pods, 0, 0);
        }
    }
    K10S_UNROLL
    for (int j = 0; j < K10S_TILE; j++) {
        bs[j] = -__builtin_inf();
        bn[j] = -1;
    }
    ulonglong2 x[2];
    tile_load(x, s_node, n_nodes, l4);
    for (uint32_t base = 0; base < n_nodes; base += 256) {
        const TileGrp g = tile_convert(x);
        tile_load(x, s_node, n_nodes, base + 256u + l4);
        const uint32_t b = tile_bits(base + l4, n_nodes);
        K10S_UNROLL
        for (int j = 0; j < K10S_TILE; j++) {
            if (!((need >> j) & 1u)) continue;   // wave-uniform
            tile_best_grp(g, b, s_node, base + l4, q[j], bs[j], bn[j]);
        }
    }
}
// The rescan of the flagged lanes' shares for one pod under the current cache (the other lanes keep
// their values); returns the entries read, summed over the wave.  Four 256-node steps per round trip.
K10S_D uint32_t tile_lane_rescan(NodeCachePtr s_node, uint32_t n_nodes, bool flag, const TileReq& q, double& bs,
                                 int32_t& bn) {
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    uint32_t nread = 0;
    if (flag) {
        bs = -__builtin_inf();
        bn = -1;
    }
    for (uint32_t base = 0; base < n_nodes; base += 1024) {
        if (flag) {
            ulonglong2 x[4][2];
            K10S_UNROLL
            for (int i = 0; i < 4; i++) tile_load(x[i], s_node, n_nodes, base + 256u * i + l4);
            K10S_UNROLL
            for (int i = 0; i < 4; i++) {
                const uint32_t n0 = base + 256u * i + l4;
                const uint32_t b = tile_bits(n0, n_nodes);
                nread += (uint32_t)__builtin_popcount(b);
                tile_best_grp(tile_convert(x[i]), b, s_node, n0, q, bs, bn);
            }
        }
    }
    return uniform_u32(wave_sum_u32(nread));
}
#else
// Host form of the pass and the rescan, the 64 lanes simulated: for every lane L of lanes, (key, idx)
// := the (score_key, index) maximum over the nodes of S_L that fit (rc, rr), idx -1 if none.
// Returns the entries read (those of the lanes scanned).
K10S_HD uint32_t tile_lanes_host(const uint64_t* s_node, uint32_t n_nodes, uint32_t rc, uint64_t rr, uint64_t lanes,
                                 uint64_t* key, int32_t* idx) {
    for (int L = 0; L < 64; L++)
        if ((lanes >> L) & 1ull) {
            key[L] = 0;
            idx[L] = -1;
        }
    uint32_t nread = 0;
    for (uint32_t n = 0; n < n_nodes; n++) {
        const uint32_t L = (n >> 2) & 63u;
        if (!((lanes >> L) & 1ull)) continue;
        nread += 1;
        const NcEnt v = nc_unpack(s_node[n]);
        if (rc <= v.cpu && rr <= v.ram) {
            const uint64_t k = score_key(la_score(v.cpu, v.ram, rc, rr));
            if (k >= key[L] || idx[L] < 0) {
                key[L] = k;
                idx[L] = (int32_t)n;
            }
        }
    }
    return nread;
}
#endif

// ---- scheduling cycle (scheduler.rs:246-334) ----------------------------------------------------
// The cycle runs out of line on the device: it runs once per many events, and out of line its
// attempt loop (the node scans, the queue pops) gets its own register allocation instead of sharing
// the event loop's.  With the action queue's top levels in LDS (K10S_AQ_TOP=15) that measured +1.2 %
// on C3 and +16.7 % on the backlog workload, where cycles run many attempts
// (profiles/r02_v5_knobs_ab.json).
// One iteration of the cycle's loop (scheduler.rs:270-329) for a live pod q at cycle time t, with the
// cycle's running duration and failure count.  pick: K10S_PICK_SCAN (scan the cache), K10S_PICK_NOFIT
// (a tile found no node for the pod: its attempt fails exactly as the scan would), or the node a
// tile resolved for it (exactly the scan's choice; the tile counted its reads).  Returns the node
// the pod was assigned, or -1.
#if !K10S_DEVICE && defined(K10S_PRUNE_STUDY)
// Tooling (tools/prune_study.py): how many entries an exact block-pruned scan would read, with tight
// componentwise block bounds, best-first block order, for block sizes 16..512.  Slots: [2i] entries
// read (bounds + blocks), [2i+1] blocks scanned; [12] scans; [40..43] near ties of the argmax.
extern "C" uint64_t k10s_prune_stats[48];
inline void k10s_prune_study(const uint64_t* s, uint32_t N, uint32_t rc, uint64_t rr) {
    k10s_prune_stats[12] += 1;
    for (int bi = 0; bi < 6; bi++) {
        const uint32_t B = 16u << bi, NB = (N + B - 1) / B;
        static uint64_t ub[1 << 12];
        for (uint32_t b = 0; b < NB; b++) {
            uint32_t mc = 0;
            uint64_t mr = 0;
            for (uint32_t n = b * B; n < N && n < (b + 1) * B; n++) {
                const NcEnt v = nc_unpack(s[n]);
                mc = v.cpu > mc ? v.cpu : mc;
                mr = v.ram > mr ? v.ram : mr;
            }
            ub[b] = (mc >= rc && mr >= rr) ? score_key(la_score(mc, mr, rc, rr)) : 0;
        }
        uint64_t best_key = 0;
        int64_t best_n = -1;
        uint64_t reads = NB, blocks = 0;
        for (;;) {
            uint64_t k = 0;
            int64_t b = -1;
            for (uint32_t x = 0; x < NB; x++)
                if (ub[x] && ub[x] >= k) {
                    k = ub[x];
                    b = x;
                }
            if (b < 0) break;
            if (best_n >= 0 && (k < best_key || (k == best_key && (int64_t)((b + 1) * B) <= best_n))) break;
            for (uint32_t n = (uint32_t)b * B; n < N && n < ((uint32_t)b + 1) * B; n++) {
                const NcEnt v = nc_unpack(s[n]);
                if (rc <= v.cpu && rr <= v.ram) {
                    const uint64_t kk = score_key(la_score(v.cpu, v.ram, rc, rr));
                    if (kk > best_key || (kk == best_key && (int64_t)n > best_n)) {
                        best_key = kk;
                        best_n = n;
                    }
                }
            }
            reads += B;
            blocks += 1;
            ub[b] = 0;
        }
        k10s_prune_stats[2 * bi] += reads;
        k10s_prune_stats[2 * bi + 1] += blocks;
    }
    // the index-aware Pareto front: nodes not weakly dominated (cpu and ram both >=) by a later node
    // — the only possible last maxima for any request; [44] its size summed over scans
    {
        std::vector<std::pair<uint32_t, uint64_t>> stair;   // seen (cpu, max ram at >= cpu), cpu descending
        uint64_t front = 0;
        for (uint32_t n = N; n-- > 0;) {
            const NcEnt v = nc_unpack(s[n]);
            if (v.cpu == 0 && v.ram == 0) continue;
            bool dom = false;
            for (const auto& p : stair) {
                if (p.first < v.cpu) break;
                if (p.second >= v.ram) {
                    dom = true;
                    break;
                }
            }
            if (dom) continue;
            front += 1;
            // insert (cpu, ram) keeping cpu descending with ram the running max
            std::vector<std::pair<uint32_t, uint64_t>> nx;
            bool put = false;
            for (const auto& p : stair) {
                if (!put && p.first <= v.cpu) {
                    nx.push_back({v.cpu, v.ram});
                    put = true;
                }
                if (p.first < v.cpu && p.second <= v.ram) continue;   // now dominated in the staircase
                if (p.first == v.cpu) continue;
                nx.push_back(p);
            }
            if (!put) nx.push_back({v.cpu, v.ram});
            uint64_t mx = 0;
            for (auto& p : nx) {
                mx = p.second > mx ? p.second : mx;
                p.second = mx;
            }
            stair.swap(nx);
        }
        k10s_prune_stats[44] += front;
    }
    // per 64-node block: its own index-aware front (within the block); [45] sum of sizes, [46] blocks
    // with more than 8, [47] the largest seen
    for (uint32_t b = 0; b * 64 < N; b++) {
        uint32_t cnt = 0;
        const uint32_t hi = (b + 1) * 64 < N ? (b + 1) * 64 : N;
        for (uint32_t k = b * 64; k < hi; k++) {
            const NcEnt v = nc_unpack(s[k]);
            if (v.cpu == 0 && v.ram == 0) continue;
            bool dom = false;
            for (uint32_t m = k + 1; m < hi && !dom; m++) {
                const NcEnt w = nc_unpack(s[m]);
                dom = w.cpu >= v.cpu && w.ram >= v.ram;
            }
            cnt += dom ? 0 : 1;
        }
        k10s_prune_stats[45] += cnt;
        k10s_prune_stats[46] += cnt > 8 ? 1 : 0;
        if (cnt > k10s_prune_stats[47]) k10s_prune_stats[47] = cnt;
    }
    // near ties of the argmax: nodes with exactly its score, within 1e-5 of its u, within 1e-4
    uint64_t bk = 0;
    for (uint32_t n = 0; n < N; n++) {
        const NcEnt v = nc_unpack(s[n]);
        if (rc <= v.cpu && rr <= v.ram) {
            const uint64_t k = score_key(la_score(v.cpu, v.ram, rc, rr));
            bk = k > bk ? k : bk;
        }
    }
    if (!bk) return;
    double bs = 0;
    for (uint32_t n = 0; n < N; n++) {
        const NcEnt v = nc_unpack(s[n]);
        if (rc <= v.cpu && rr <= v.ram && score_key(la_score(v.cpu, v.ram, rc, rr)) == bk) bs = la_score(v.cpu, v.ram, rc, rr);
    }
    for (uint32_t n = 0; n < N; n++) {
        const NcEnt v = nc_unpack(s[n]);
        if (!(rc <= v.cpu && rr <= v.ram)) continue;
        const double sc = la_score(v.cpu, v.ram, rc, rr);
        const double du = (bs - sc) * 0.02;
        if (sc == bs) k10s_prune_stats[40] += 1;
        if (du <= 1e-5) k10s_prune_stats[41] += 1;
        if (du <= 1e-4) k10s_prune_stats[42] += 1;
        if (du <= 1e-3) k10s_prune_stats[43] += 1;
    }
}
// Cycle depth study: the cache at the cycle's start (snapshot) and the nodes reserved so far in
// the cycle; for each attempt, d = 1 + the number of reserved nodes whose snapshot (score, index)
// beats the pod's pick in the snapshot order — the depth a per-pod snapshot top-K list needs.
// Histogram slots [16 + min(d, 15)]; [13] cycles, [14] attempts in cycles, [15] distinct reserved.
struct PruneCyc {
    std::vector<uint64_t> snap;
    std::vector<uint32_t> rset;
};
inline PruneCyc& prune_cyc() {
    static PruneCyc p;
    return p;
}
inline void k10s_prune_cycle_start(const uint64_t* s, uint32_t N) {
    PruneCyc& p = prune_cyc();
    p.snap.assign(s, s + N);
    p.rset.clear();
    k10s_prune_stats[13] += 1;
}
inline void k10s_prune_cycle_pick(uint32_t rc, uint64_t rr, int32_t pick) {
    PruneCyc& p = prune_cyc();
    k10s_prune_stats[14] += 1;
    if (pick < 0) return;
    // pick's snapshot key
    auto key = [&](uint32_t n) -> uint64_t {
        const NcEnt v = nc_unpack(p.snap[n]);
        return (rc <= v.cpu && rr <= v.ram) ? score_key(la_score(v.cpu, v.ram, rc, rr)) : 0;
    };
    // the best snapshot node outside the reserved set, then the reserved nodes above it
    std::vector<char> inr(p.snap.size(), 0);
    for (uint32_t n : p.rset) inr[n] = 1;
    uint64_t kp = 0;
    int64_t m = -1;
    for (uint32_t n = 0; n < p.snap.size(); n++) {
        if (inr[n]) continue;
        const uint64_t k = key(n);
        if (k && (k > kp || (k == kp && (int64_t)n > m))) {
            kp = k;
            m = n;
        }
    }
    uint32_t d = 1;
    for (uint32_t n : p.rset) {
        const uint64_t k = key(n);
        if (k > kp || (k == kp && (int64_t)n > m)) d++;
    }
    k10s_prune_stats[16 + (d < 15 ? d : 15)] += 1;
    bool seen = false;
    for (uint32_t n : p.rset) seen |= n == (uint32_t)pick;
    if (!seen) {
        p.rset.push_back((uint32_t)pick);
        k10s_prune_stats[15] += 1;
    }
}
#endif
#define K10S_PICK_SCAN (-1)
#define K10S_PICK_NOFIT (-2)
#define K10S_PICK_PRUNED (-3)   // the tile's block bounds are valid: tile_scan_pruned (TILE builds only)
template <bool PLUG, bool TILE = false>
K10S_HD int32_t cycle_attempt(Ctx& c, double t, QInfo q, int32_t pick, double& cycle_dur, uint32_t& fails) {
    RepHdr* h = &c.H();
    const double w = c.P().score_weight;
    const uint32_t p = q.pod;
    const double queue_t = t - q.initial + cycle_dur;
    const uint32_t nn = h->s_node_count;
    const double sched_time = 0.000001 * (double)nn;  // ConstantTimePerNodeModel (model.rs:24-26)
    cycle_dur += sched_time;
    const uint32_t rc = c.V().pod(p).req_cpu;
    const uint64_t rr = c.V().pod(p).req_ram;
    int st;
    int32_t chosen = -1;
    if (rc == 0 && rr == 0) {
        st = K10S_SCHED_REQUESTED_RESOURCES_ARE_ZEROS;
    } else if (nn == 0) {
        st = K10S_SCHED_NO_NODES_IN_CLUSTER;
    } else {
        h->counters[K10S_C_ATTEMPTS] += 1;
        h->counters[K10S_C_NODES_SCANNED] += nn;
        st = -1;
        uint32_t nread = 0;
        const uint64_t t_scan = prof_now();
        if (pick == K10S_PICK_NOFIT) {
            st = K10S_SCHED_NO_SUFFICIENT_RESOURCES;   // (the tile's pass counted its reads)
        } else if (pick >= 0) {
            st = K10S_SCHED_OK;
            chosen = pick;
        } else if (TILE && pick == K10S_PICK_PRUNED) {
            uint32_t pr = 0;
            st = tile_scan_pruned(c.V().s_node(), c.V().s_bram(), c.S().n_nodes, c.Ly().bshift, rc, rr, &chosen, &pr);
            nread = pr;
        } else if (PLUG) {
            st = schedule_scan_plugins(c, rc, rr, &chosen);
            nread = c.S().n_nodes;
        } else if (!nc_packed(c) && c.Ly().pruned && w == 1.0 && rc > 0 && rr > 0) {
            st = schedule_scan_pruned(c, rc, rr, &chosen, &nread);
        }
        // fronts in the serial cycle only: a tile's cycle (after failed attempts) places few pods, and
        // rebuilding the blocks that the finishes since the last cycle marked would cost more than
        // its full scans (backlog +9 %, profiles/r06_g6_fronts_ab.json)
        if (st < 0 && K10S_FRONT && !PLUG && !TILE && c.Ly().front && w == 1.0 && rc > 0 && rr > 0) {
            nread += fr_refresh(c);
            uint32_t fr = 0;
            st = front_scan(c, rc, rr, &chosen, &fr);
            nread += fr;
        }
        if (st < 0) {
#if !K10S_DEVICE && defined(K10S_PRUNE_STUDY)
            if (nc_packed(c) && w == 1.0 && rc > 0 && rr > 0) k10s_prune_study(c.V().s_node(), c.S().n_nodes, rc, rr);
#endif
            if (nc_packed(c))
                st = schedule_scan<true, true>(nullptr, c.V().s_node(), c.V().s_present(), c.S().n_nodes, rc, rr, w,
                                               &chosen);
            else
                st = schedule_scan<true, false>(c.V().s_cpu(), c.V().s_ram(), c.V().s_present(), c.S().n_nodes, rc, rr,
                                                w, &chosen);
            nread += c.S().n_nodes;   // (after a pruned scan that gave up: its reads too)
        }
        h->counters[K10S_C_NODES_READ] += nread;
        K10S_PROF_ADD(c, PROF_SCAN, t_scan);
        K10S_PROF_COUNT(c, PROF_NSCAN);
    }
    if (st != K10S_SCHED_OK) {
        fails += 1;
        q.timestamp = t + cycle_dur;
        uq_insert(c, q);
        emit(c, K10S_EV_AS_POD_NOT_SCHEDULED, c.P().sched_to_as_network_delay, -1, p, 0, t + cycle_dur, FQ_SCHED_TO_AS);
        return -1;
    }
    const uint32_t n = (uint32_t)chosen;
    nc_reserve(c, n, rc, rr);  // reserve_node_resources (118-123)
    node_bound_changed(c, n);
    c.V().node(n).flags |= NF_S_ASSIGN;  // assign_node_to_pod (125-151)
    c.V().pod(p).s_assigned = (int32_t)n;
    emit(c, K10S_EV_AS_ASSIGN_REQ, cycle_dur + c.P().sched_to_as_network_delay, -1, p, n, t + cycle_dur, FQ_ASSIGN);
    h->counters[K10S_C_PLACEMENTS] += 1;
    if (c.V().place()) {
        const uint32_t k = h->place_n;
        if (k < c.Ly().cap_place) {
            c.V().place()[k].assign_time = t + cycle_dur;
            c.V().place()[k].pod = (int32_t)p;
            c.V().place()[k].node = (int32_t)n;
            h->place_n = k + 1;
        } else {
            h->flags |= 2u;
        }
    }
    est_add(h->est[K10S_EST_POD_SCHEDULE_TIME], sched_time);
    est_add(h->est[K10S_EST_POD_QUEUE_TIME], queue_t);
    return (int32_t)n;
}
// The end of a cycle: the next one after max(its duration, the interval) (scheduler.rs:331-333).
K10S_HD void cycle_end(Ctx& c, double cycle_dur, uint32_t fails) {
    c.H().cyc_fails = fails;
    emit0(c, K10S_EV_S_RUN_CYCLE, fmax_rs(cycle_dur, c.P().scheduling_cycle_interval));
}

template <bool PLUG>
K10S_HD_NOINL void run_scheduling_cycle_t(Ctx& c, double t) {
    if (!K10S_FULL_WAVE(XG_CYCLE)) return;
    double cycle_dur = 0.0;
    uint32_t fails = 0;
    RepHdr* h = &c.H();
    h->g_pods_q = (uint64_t)h->aq_size + (uint64_t)h->uq_size;  // scheduler.rs:256-259
#if !K10S_DEVICE && defined(K10S_PRUNE_STUDY)
    if (nc_packed(c)) k10s_prune_cycle_start(c.V().s_node(), c.S().n_nodes);
#endif
    while (c.H().aq_size > 0 && !c.H().error_code) {
        const uint64_t t_aq = prof_now();
        const QInfo q = aq_pop(c);
        K10S_PROF_ADD(c, PROF_AQPOP, t_aq);
        if (!pod_in_s(c, q.pod)) continue;   // removed from the cache (scheduler.rs:263-269)
#if !K10S_DEVICE && defined(K10S_PRUNE_STUDY)
        const int32_t placed =
#endif
        cycle_attempt<PLUG>(c, t, q, K10S_PICK_SCAN, cycle_dur, fails);
#if !K10S_DEVICE && defined(K10S_PRUNE_STUDY)
        if (nc_packed(c)) k10s_prune_cycle_pick(c.V().pod(q.pod).req_cpu, c.V().pod(q.pod).req_ram, placed);
#endif
    }
    cycle_end(c, cycle_dur, fails);
}

// The cycle in tiles (fit_tile above): run after a cycle with failed attempts, on the
// LeastAllocated-only fast path with the packed cache (its own out-of-line function, so the serial
// cycle's register allocation is unchanged).  The next K10S_TILE entries are popped in order (the
// same pops the loop would make) and kept in the queue array slots their pops vacated (slot top-1-j
// for the j-th: the array only shrinks during a cycle; HBM part), a removed pod marked and later
// skipped like the loop's `continue`; their fit is tested together, then each is attempted in order.
// Error state: a capacity error (QUEUE_FULL / HEAP_FULL) mid-tile drops the tile's unattempted
// entries, so aq_size / active_len of an errored replica is unspecified (the serial cycle would stop
// popping one entry earlier); an errored replica's results are refused anyway.
K10S_HD_NOINL void run_scheduling_cycle_tiles(Ctx& c, double t) {
    if (!K10S_FULL_WAVE(XG_CYCLE)) return;
    double cycle_dur = 0.0;
    uint32_t fails = 0;
    RepHdr* h = &c.H();
    h->g_pods_q = (uint64_t)h->aq_size + (uint64_t)h->uq_size;  // scheduler.rs:256-259
    while (c.H().aq_size > 0 && !c.H().error_code) {
        // the tile's j-th pop is kept in the HBM slot its pop vacated: the array's end (heap) or its own
        // position (sorted mode, aq_pop: the front); HBM slots below K10S_AQ_TOP are otherwise unused
        const bool srt = uniform_u32(h->aq_sorted) != 0u;
        const uint32_t top = uniform_u32(h->aq_size);
        QInfo* slot = c.V().aq() + (srt ? uniform_u32(h->aq_head) : top - 1u);
        const int32_t sdir = srt ? 1 : -1;
        uint32_t nt = 0;
        const uint64_t t_aq = prof_now();
        for (; nt < K10S_TILE && c.H().aq_size > 0; nt++) {
            QInfo q = aq_pop(c);
            if (!pod_in_s(c, q.pod)) q.pod = 0xFFFFFFFFu;
            slot[sdir * (int32_t)nt] = q;
        }
        K10S_PROF_ADD(c, PROF_AQPOP, t_aq);
        wave_sync();
        // the tile's requests (fast-path pods only: both requests > 0 and within the packed fields;
        // a request beyond them fits no packed entry)
        uint32_t rc8[K10S_TILE];
        uint64_t rrq[K10S_TILE];
        uint32_t need = 0, never = 0;
        K10S_UNROLL
        for (int j = 0; j < K10S_TILE; j++) {
            rc8[j] = 0xFFFFFFFFu;
            rrq[j] = ~0ull;
            if ((uint32_t)j < nt) {
                const uint32_t p = uniform_u32(slot[sdir * j].pod);
                if (p != 0xFFFFFFFFu) {
                    const uint32_t rc = uniform_u32(c.V().pod(p).req_cpu);
                    const uint64_t rr = uniform_u64(c.V().pod(p).req_ram);
                    if (rc > 0 && rr > 0) {
                        if (rc <= K10S_PK_CPU && rr <= K10S_PK_RAM) {
                            rc8[j] = rc << 8;
                            rrq[j] = rr;
                            need |= 1u << j;
                        } else {
                            never |= 1u << j;
                        }
                    }
                }
            }
        }
        uint32_t found = 0;
        const uint64_t* s_node = c.V().s_node();
        const uint32_t N = c.S().n_nodes;
#if K10S_TILE_BEST
        // b_jL of every pod of need (device: lane L's own registers; host: the lanes simulated)
#if K10S_DEVICE
        double tbs[K10S_TILE];
        int32_t tbn[K10S_TILE];
#else
        uint64_t tbk[K10S_TILE][64];
        int32_t tbn[K10S_TILE][64];
#endif
        if (need && h->s_node_count > 0) {
            const uint64_t t_fit = prof_now();
#if K10S_DEVICE
            tile_best_pass((NodeCachePtr)s_node, N, (K10S_GB(const QInfo))slot, sdir,
                           (K10S_GB(const PodState))&c.V().pod(0), need, tbs, tbn);
            K10S_UNROLL
            for (int j = 0; j < K10S_TILE; j++)
                if (__ballot(tbn[j] >= 0)) found |= 1u << j;
#else
            for (int j = 0; j < K10S_TILE; j++) {   // (one shared read on the device)
                if (!((need >> j) & 1u)) continue;
                tile_lanes_host(s_node, N, rc8[j] >> 8, rrq[j], ~0ull, tbk[j], tbn[j]);
                for (int L = 0; L < 64; L++)
                    if (tbn[j][L] >= 0) found |= 1u << j;
            }
#endif
            h->counters[K10S_C_NODES_READ] += N;
            K10S_PROF_ADD(c, PROF_SCAN, t_fit);
        }
#else
        // block bounds for the pods that fit (tile_scan_pruned): blocks of 64..256 nodes
        const uint32_t bsh = c.Ly().bshift;
        const bool bounds = K10S_TILE_PRUNE && bsh <= 8;
        if (need && h->s_node_count > 0) {
            uint32_t nread = 0;
            const uint64_t t_fit = prof_now();
            found = fit_tile(s_node, N, rc8, rrq, need, &nread, bounds ? c.V().s_bram() : nullptr, bsh);
            h->counters[K10S_C_NODES_READ] += nread;
            K10S_PROF_ADD(c, PROF_SCAN, t_fit);
        }
#endif
        const uint32_t nofit = (need & ~found) | never;
        [[maybe_unused]] uint64_t rlanes = 0;   // lanes whose share holds a node reserved by this tile
        for (uint32_t j = 0; j < nt && !c.H().error_code; j++) {
            const QInfo q = slot[sdir * (int32_t)j];
            if (uniform_u32(q.pod) == 0xFFFFFFFFu) continue;
            QInfo u;
            u.timestamp = uniform_f64(q.timestamp);
            u.initial = uniform_f64(q.initial);
            u.attempts = uniform_u32(q.attempts);
            u.pod = uniform_u32(q.pod);
            int32_t pick = (nofit >> j) & 1u ? K10S_PICK_NOFIT : K10S_PICK_SCAN;
#if !K10S_TILE_BEST
            if (bounds && ((need & found) >> j & 1u)) pick = K10S_PICK_PRUNED;
#endif
#if K10S_TILE_BEST
            if ((found >> j) & 1u) {   // fits some node of the snapshot: resolve from the lane values
                const uint64_t t_pick = prof_now();
                const uint32_t rc = uniform_u32(c.V().pod(u.pod).req_cpu);
                const uint64_t rr = uniform_u64(c.V().pod(u.pod).req_ram);
#if K10S_DEVICE
                double s = tbs[j];
                int32_t n = tbn[j];
                if (rlanes) {
                    const bool flag = (rlanes >> lane_id()) & 1ull;
                    h->counters[K10S_C_NODES_READ] += tile_lane_rescan((NodeCachePtr)s_node, N, flag,
                                                                   tile_req((K10S_GB(const PodState))&c.V().pod(u.pod), rc, rr), s, n);
                }
                uint64_t key = n >= 0 ? score_key(s) : 0;
                wave_argmax(key, n);
                n = (int32_t)uniform_u32((uint32_t)n);
#else
                if (rlanes) h->counters[K10S_C_NODES_READ] += tile_lanes_host(s_node, N, rc, rr, rlanes, tbk[j], tbn[j]);
                uint64_t key = 0;
                int32_t n = -1;
                for (int L = 0; L < 64; L++)
                    if (tbn[j][L] >= 0 && (tbk[j][L] > key || (tbk[j][L] == key && tbn[j][L] > n))) {
                        key = tbk[j][L];
                        n = tbn[j][L];
                    }
                K10S_HSTAT(HS_TILE_PICKS);
                if (rlanes) K10S_HSTAT(HS_TILE_RESCANS);
#endif
                pick = n >= 0 ? n : K10S_PICK_NOFIT;
#if !K10S_DEVICE && defined(K10S_TILE_DEBUG)
                {
                    int32_t ch = -1;
                    const int st = schedule_scan<true, true>(nullptr, s_node, c.V().s_present(), N, rc, rr, 1.0, &ch);
                    const int32_t want = st == K10S_SCHED_OK ? ch : K10S_PICK_NOFIT;
                    if (want != pick) {
                        fprintf(stderr, "TILE MISMATCH t=%.6f pod=%u j=%u pick=%d scan=%d rlanes=%llx nt=%u\n", t, u.pod, j, pick, want,
                                (unsigned long long)rlanes, nt);
                        for (uint32_t m = 0; m < N; m++) {
                            const NcEnt v = nc_unpack(s_node[m]);
                            fprintf(stderr, "  node %u cpu=%u ram=%llu pres=%d\n", m, v.cpu, (unsigned long long)v.ram,
                                    (int)((c.V().s_present()[m >> 6] >> (m & 63)) & 1));
                        }
                        fprintf(stderr, "  rc=%u rr=%llu\n", rc, (unsigned long long)rr);
                    }
                }
#endif
                K10S_PROF_ADD(c, PROF_SCAN, t_pick);
            }
#endif
            // every assignment of the tile marks its lane (a pod outside need, e.g. one zero
            // request, is placed by the scan and changes the cache too)
            const int32_t placed = cycle_attempt<false, true>(c, t, u, pick, cycle_dur, fails);
            if (placed >= 0) rlanes |= 1ull << (((uint32_t)placed >> 2) & 63u);
        }
    }
    cycle_end(c, cycle_dur, fails);
}

// ---- pods of a node in name order (wave ballot over pod indices) ---------------------------------
// Calls f(p) for every pod p (ascending) with pred(p); stops early if c.H().error_code.
template <typename Pred, typename F>
K10S_HD void for_each_pod_in_order(Ctx& c, Pred pred, F f) {
    if (!K10S_FULL_WAVE(XG_PODS_IN_ORDER)) return;
    const uint32_t P = c.S().n_pods;
    for (uint32_t base = 0; base < P; base += K10S_LANES) {
        uint32_t p = base + (uint32_t)lane_id();
        bool m = p < P && pred(p);
#if K10S_DEVICE
        uint64_t mask = __ballot(m);
        while (mask) {
            uint32_t b = (uint32_t)__builtin_ctzll(mask);
            mask &= mask - 1;
            f(base + b);
            if (c.H().error_code) return;
        }
#else
        if (m) {
            f(p);
            if (c.H().error_code) return;
        }
#endif
    }
}

// ---- scheduler handlers (scheduler.rs:382-477) ---------------------------------------------------
K10S_HD void s_release(Ctx& c, uint32_t p) {  // release_node_resources (153-162)
    int32_t n = c.V().pod(p).s_assigned;
    if (n < 0 || !bit_test(c.V().s_present(), (uint32_t)n)) {
        fail(c, K10S_PANIC_MISSING_NODE);
        return;
    }
    if (!nc_release(c, (uint32_t)n, nc_get(c, (uint32_t)n), c.V().pod(p).req_cpu, c.V().pod(p).req_ram)) return;
    node_bound_changed(c, (uint32_t)n);
}

// K10S_TILE_ALWAYS=1: every LeastAllocated-only cycle on the packed cache runs in tiles (A/B knob).
#ifndef K10S_TILE_ALWAYS
#define K10S_TILE_ALWAYS 0
#endif
K10S_HD void run_scheduling_cycle(Ctx& c, double t) {
    if (nc_packed(c) && c.P().score_weight == 1.0 && (K10S_TILE_ALWAYS || c.H().cyc_fails != 0))
        run_scheduling_cycle_tiles(c, t);
    else run_scheduling_cycle_t<false>(c, t);
}
// A replica whose profile is not LeastAllocated alone (K10S_SCORE_PLUGINS builds only: the host
// engine and k10s_kernels_plugins.hip; compiled into the default kernel, the branch alone cost
// 4.6 % at C3, profiles/r02_v4_score_plugins_ab.json).
K10S_HD void run_scheduling_cycle_plugins(Ctx& c, double t) { run_scheduling_cycle_t<true>(c, t); }

// AddNodeToCache (scheduler.rs:391-405)
K10S_HD void s_add_node(Ctx& c, const HeapEv& e) {
    RepHdr* h = &c.H();
    uint32_t n = e.a;
    uint32_t ac = e.b;
    uint64_t ar = f2u(e.x);
    const NcEnt cap = {ac, ar};
    nc_put(c, n, cap);
    fr_mark(c, n);
    // the stored node's capacity: a node reaches the scheduler straight from its creation,
    // allocatable = capacity (node.rs:60-66); only MostAllocated reads it (wide layout)
    if (!nc_packed(c)) {
        c.V().s_ccpu()[n] = ac;
        c.V().s_cram()[n] = ar;
    }
    if (!bit_test(c.V().s_present(), n)) {
        bit_set(c.V().s_present(), n);
        h->s_node_count += 1;
    }
    node_bound_changed(c, n);
    if (c.P().enable_unscheduled_pods_conditional_move) s_move(c, 3, 0.0, ac, ar);
    else s_move(c, 0, 0.0, 0, 0);
}
// PodScheduleRequest (scheduler.rs:411-420)
K10S_HD void s_pod_schedule_req(Ctx& c, const HeapEv& e) {
    uint32_t p = e.a;
    c.V().pod(p).sflag = PF_IN_S;   // a store: no read of the pod line on this event
    c.V().pod(p).s_assigned = -1;
    QInfo q;
    q.timestamp = e.time;
    q.initial = e.time;
    q.attempts = 1;
    q.pod = p;
    aq_push(c, q);
}
K10S_HD void on_scheduler(Ctx& c, const HeapEv& e) {
    RepHdr* h = &c.H();
    switch (e.kind) {
    case K10S_EV_S_RUN_CYCLE: {
        const uint64_t t0 = prof_now();
        if (K10S_SCORE_PLUGINS && c.P().score_plugins != K10S_SCORE_LEAST_ALLOCATED) run_scheduling_cycle_plugins(c, e.time);
        else run_scheduling_cycle(c, e.time);
        K10S_PROF_ADD(c, PROF_CYCLE, t0);
        break;
    }
    case K10S_EV_S_FLUSH:
        s_move(c, 1, e.time, 0, 0);
        emit0(c, K10S_EV_S_FLUSH, 30.0);  // POD_FLUSH_INTERVAL (queue.rs:11)
        break;
    case K10S_EV_S_ADD_NODE:
        s_add_node(c, e);
        break;
    case K10S_EV_S_POD_SCHEDULE_REQ:
        s_pod_schedule_req(c, e);
        break;
    case K10S_EV_S_POD_FINISHED: {
        uint32_t p = e.a, n = e.b;
        // one batch of loads: the pod's fields, the event node's flags, and the scheduler-cache entry
        // of the event node (the pod's assigned node in every run so far; re-read if it is not)
        PodState& P = c.V().pod(p);
        const uint8_t pf = P.sflag;
        const int32_t sa = P.s_assigned;
        const uint32_t rc = P.req_cpu;
        const uint64_t rr = P.req_ram;
        const uint8_t nf = c.V().node(n).flags;
        const bool n_present = bit_test(c.V().s_present(), n);
        const NcEnt nv = nc_get(c, n);
        if (!(pf & PF_IN_S)) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        P.sflag = 0;
        if (!(nf & NF_S_ASSIGN)) {
            fail(c, K10S_PANIC_MISSING_ASSIGNMENTS);
            return;
        }
        // release_node_resources (scheduler.rs:153-162) on the pod's assigned node
        const bool present = sa == (int32_t)n ? n_present : (sa >= 0 && bit_test(c.V().s_present(), (uint32_t)sa));
        if (sa < 0 || !present) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        if (!nc_release(c, (uint32_t)sa, sa == (int32_t)n ? nv : nc_get(c, (uint32_t)sa), rc, rr)) return;
        node_bound_changed(c, (uint32_t)sa);
        s_move_after_free(c, rc, rr);
        break;
    }
    case K10S_EV_S_REMOVE_NODE: {
        uint32_t n = e.a;
        if (!bit_test(c.V().s_present(), n)) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        bit_clear(c.V().s_present(), n);
        // invariant: an absent node's cache entry is (0, 0), as after initialize, so no request with
        // cpu > 0 fits it and the event loop's screened scan needs no presence words
        const NcEnt zero = {0u, 0ull};
        nc_put(c, n, zero);
        fr_mark(c, n);
        h->s_node_count -= 1;
        node_bound_changed(c, n);
        if (c.V().node(n).flags & NF_S_ASSIGN) {  // reschedule_unfinished_pods (352-364), name order
            c.V().node(n).flags &= (uint8_t)~NF_S_ASSIGN;
            double t = e.time;
            for_each_pod_in_order(
                c, [&](uint32_t p) { return pod_in_s(c, p) && c.V().pod(p).s_assigned == (int32_t)n; },
                [&](uint32_t p) {
                    c.V().pod(p).s_assigned = -1;
                    QInfo q;
                    q.timestamp = t;
                    q.initial = t;
                    q.attempts = 1;
                    q.pod = p;
                    aq_push(c, q);
                });
        }
        break;
    }
    case K10S_EV_S_REMOVE_POD: {
        uint32_t p = e.a;
        if (!pod_in_s(c, p)) return;
        c.V().pod(p).sflag = 0;
        int32_t n = c.V().pod(p).s_assigned;
        if (n >= 0) {
            s_release(c, p);
            if (c.H().error_code) return;
            if (!(c.V().node(n).flags & NF_S_ASSIGN)) {
                fail(c, K10S_PANIC_MISSING_ASSIGNMENTS);
                return;
            }
            s_move_after_free(c, c.V().pod(p).req_cpu, c.V().pod(p).req_ram);
        }
        break;
    }
    default:
        break;
    }
}

// ---- cluster autoscaler decision (kube_cluster_autoscaler.rs) -----------------------------------
// Computed when persistent storage builds the Auto info (persistent_storage.rs:381-412): the
// info is a snapshot of PS state at that instant, and the CA's node-group state is only touched
// by autoscale() while exactly one request is in flight, so deciding at snapshot time and
// emitting the actions at delivery time (cluster_autoscaler.rs:309-331) is equivalent.
//
// Lane-parallel where the reference loops over collections: the unscheduled-pod cache and the
// CA-origin nodes are bitmaps read 64 words per step (set bits visited in ascending index = name
// order), a node's assigned pods come from its PS assignment list (O(pods on the node), then sorted
// by name), and every first-fit over nodes is a wave "lowest fitting index" over 4-node lane groups.
// The serial parts are the reference's own sequential dependences (each placement changes the
// allocatable the next pod sees).

// Calls f(i) for every set bit i of words[0, W) in ascending order; stops early on an error.
template <typename F>
K10S_HD void for_each_bit(Ctx& c, const uint64_t* words, uint32_t W, F f) {
    if (!K10S_FULL_WAVE(XG_FOR_EACH_BIT)) return;
    for (uint32_t wb = 0; wb < W; wb += K10S_LANES) {
        const uint32_t w = wb + (uint32_t)lane_id();
        const uint64_t word = w < W ? words[w] : 0ull;
#if K10S_DEVICE
        uint64_t nz = __ballot(word != 0);
        while (nz) {
            const uint32_t l = (uint32_t)__builtin_ctzll(nz);
            nz &= nz - 1;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)word, (int)l);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(word >> 32), (int)l);
            uint64_t bits = (uint64_t)lo | ((uint64_t)hi << 32);
            while (bits) {
                const uint32_t b = (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                f((wb + l) * 64u + b);
                if (c.H().error_code) return;
            }
        }
#else
        uint64_t bits = word;
        while (bits) {
            const uint32_t b = (uint32_t)__builtin_ctzll(bits);
            bits &= bits - 1;
            f(w * 64u + b);
            if (c.H().error_code) return;
        }
#endif
    }
}

// Lowest index m in [0, n), m != skip, with rc <= ca_cpu[m] && rr <= ca_ram[m]; -1 if none.
// (node_fits_pod, kube_cluster_autoscaler.rs:82-85, as the first-fit loops 114-123 / 159-178 use it.)
K10S_HD int32_t ca_first_fit(Ctx& c, uint32_t n, uint32_t skip, uint32_t rc, uint64_t rr) {
    const uint32_t* cc = c.V().ca_cpu();
    const uint64_t* cr = c.V().ca_ram();
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_CA_FIRST_FIT)) return -1;
    // each lane tests 4 consecutive entries per 256-entry step (one 16-B cpu load, two 16-B ram
    // loads: the sections are 256-B aligned and padded, entries >= n are masked out)
    const uint32_t l4 = 4u * (uint32_t)lane_id();
    for (uint32_t base = 0; base < n; base += 256) {
        const uint32_t m0 = base + l4;
        uint32_t bits = 0;
        if (m0 < n) {
            const uint4 cv = *reinterpret_cast<const uint4*>(cc + m0);
            const ulonglong2 r01 = *reinterpret_cast<const ulonglong2*>(cr + m0);
            const ulonglong2 r23 = *reinterpret_cast<const ulonglong2*>(cr + m0 + 2);
            bits = (uint32_t)(rc <= cv.x && rr <= r01.x) | ((uint32_t)(rc <= cv.y && rr <= r01.y) << 1) |
                   ((uint32_t)(rc <= cv.z && rr <= r23.x) << 2) | ((uint32_t)(rc <= cv.w && rr <= r23.y) << 3);
            const uint32_t valid = n - m0;
            bits &= valid >= 4 ? 0xFu : ((1u << valid) - 1u);
            if (skip - m0 < 4u) bits &= ~(1u << (skip - m0));
        }
        const uint64_t any = __ballot(bits != 0);
        if (any) {
            const uint32_t l = (uint32_t)__builtin_ctzll(any);
            const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)bits, (int)l);
            return (int32_t)(base + 4u * l + (uint32_t)__builtin_ctz(lb));
        }
    }
    return -1;
#else
    for (uint32_t m = 0; m < n; m++)
        if (m != skip && rc <= cc[m] && rr <= cr[m]) return (int32_t)m;
    return -1;
#endif
}

// Sort the k distinct pod indices src[0, k) ascending into dst[0, k) (BTreeSet<String> order of a
// node's assignment set).  Device: rank sort, 64 elements per pass against all k.
K10S_HD void ca_sort(const uint32_t* src, uint32_t* dst, uint32_t k) {
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_CA_SORT)) return;
    const uint32_t lane = (uint32_t)lane_id();
    for (uint32_t cb = 0; cb < k; cb += 64) {
        const uint32_t mine = cb + lane < k ? src[cb + lane] : 0xFFFFFFFFu;
        uint32_t rank = 0;
        for (uint32_t ob = 0; ob < k; ob += 64) {
            const uint32_t other = ob + lane < k ? src[ob + lane] : 0xFFFFFFFFu;
            const uint32_t m = k - ob < 64u ? k - ob : 64u;
            for (uint32_t j = 0; j < m; j++)
                rank += (uint32_t)__builtin_amdgcn_readlane((int)other, (int)j) < mine ? 1u : 0u;
        }
        if (cb + lane < k) dst[rank] = mine;
    }
    wave_sync();
#else
    for (uint32_t i = 0; i < k; i++) {
        uint32_t x = src[i], j = i;
        for (; j > 0 && dst[j - 1] > x; j--) dst[j] = dst[j - 1];
        dst[j] = x;
    }
#endif
}

K10S_COLD void ca_decide(Ctx& c) {
    RepHdr* h = &c.H();
    const Scenario* sc = &c.S();
    h->ca_n_act = 0;
    uint32_t* cag = c.V().cag();
    const uint64_t max_nodes = c.P().ca_max_node_count;
    if (h->unsched_cache_count > 0) {
        // scale_up_info (persistent_storage.rs:137-145) looks every cached unscheduled pod up in
        // storage before the algorithm runs: a removed one panics (the cache is never cleaned, A.5)
        if (h->unsched_missing > 0) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        // scale_up (191-245)
        uint64_t cur = 0;
        for (uint32_t g = 0; g < sc->n_ca_groups; g++) cur += cag[2 * g];
        bool over = true;  // node_count_over_quota (62-80)
        if (cur < max_nodes) {
            for (uint32_t g = 0; g < sc->n_ca_groups; g++) {
                if (!sc->ca_has_max[g] || cag[2 * g] < sc->ca_max[g]) {
                    over = false;
                    break;
                }
            }
        }
        if (over) return;
        uint32_t nalloc = 0;
        // the unscheduled-pod cache in name order (BTreeSet, persistent_storage.rs:41)
        for_each_bit(c, c.V().ca_ubits(), c.Ly().words_pods, [&](uint32_t p) {
            const uint32_t rc = uniform_u32(c.V().pod(p).req_cpu);
            const uint64_t rr = uniform_u64(c.V().pod(p).req_ram);
            const int32_t i = ca_first_fit(c, nalloc, 0xFFFFFFFFu, rc, rr);   // try_fit_in_allocated_nodes (114-123)
            if (i >= 0) {
                c.V().ca_cpu()[i] -= rc;
                c.V().ca_ram()[i] -= rr;
                return;
            }
            if (cur >= max_nodes) return;
            for (uint32_t g = 0; g < sc->n_ca_groups; g++) {  // try_find_fitting_template (88-112)
                if (sc->ca_has_max[g] && cag[2 * g] >= sc->ca_max[g]) continue;
                if (rc <= sc->ca_cpu[g] && rr <= sc->ca_ram[g]) {
                    cag[2 * g] += 1;
                    cag[2 * g + 1] += 1;
                    const uint32_t k = cag[2 * g + 1];
                    if (k > sc->ca_bound) {
                        fail(c, K10S_ERR_NAME_BOUND);
                        return;
                    }
                    if (nalloc >= c.Ly().cap_act) {
                        fail(c, K10S_ERR_CA_BUFFER);
                        return;
                    }
                    c.V().ca_act()[nalloc].up = 1;
                    c.V().ca_act()[nalloc].arg = sc->ca_def[g * sc->ca_bound + (k - 1)];
                    c.V().ca_cpu()[nalloc] = sc->ca_cpu[g];
                    c.V().ca_ram()[nalloc] = sc->ca_ram[g];
                    wave_sync();
                    nalloc++;
                    cur++;
                    return;
                }
            }
        });
        h->ca_n_act = nalloc;
        return;
    }
    // scale_down (247-306) over the PS-present CA-origin nodes in name order.  `info.nodes` is
    // materialized lazily: until some candidate has pods to move, every node's allocatable is its
    // PS value; the first such candidate copies all of them (absent nodes as (0, 0), so they fit
    // no pod with a nonzero request) and the moves then mutate the copy (all_pods_can_be_moved_to_
    // other_nodes, 148-181).
    const uint32_t N = sc->n_nodes;
    bool copied = false;
    uint32_t nrem = 0;
    for_each_bit(c, c.V().ca_live(), c.Ly().words_nodes, [&](uint32_t n) {
        const NodeState& ND = c.V().node(n);
        const uint32_t def = uniform_u32(ND.ps_def);
        const uint32_t cap_c = sc->def_cpu[def];
        const uint64_t cap_r = sc->def_ram[def];
        const uint32_t ac = uniform_u32(copied ? c.V().ca_cpu()[n] : ND.ps_cpu);
        const uint64_t ar = uniform_u64(copied ? c.V().ca_ram()[n] : ND.ps_ram);
        const double cu = (double)(uint32_t)(cap_c - ac) / (double)cap_c;   // is_under_threshold_utilization (128-142)
        const double ru = (double)(uint64_t)(cap_r - ar) / (double)cap_r;
        const double util = cu > ru ? cu : ru;
        if (!(util < c.P().ca_scale_down_utilization_threshold)) return;
        // the node's assigned pods in name order (info.assignments[node], 271-276)
        uint32_t* gath = c.V().ca_list();
        uint32_t* sorted = gath + sc->n_pods;
        uint32_t k = 0;
        for (int32_t p = uniform_u32((uint32_t)c.V().ps_head()[n]); p >= 0;
             p = (int32_t)uniform_u32((uint32_t)c.V().ps_link()[2 * p + 1])) {
            if (k >= sc->n_pods) {   // a corrupt list would never end: impossible by construction
                fail(c, K10S_ERR_CA_BUFFER);
                return;
            }
            gath[k++] = (uint32_t)p;
        }
        wave_sync();
        if (k > 0) {
            ca_sort(gath, sorted, k);
            if (!copied) {
                for (uint32_t m = (uint32_t)lane_id(); m < N; m += K10S_LANES) {
                    const NodeState& M = c.V().node(m);
                    const bool pres = (M.flags & NF_PS_PRESENT) != 0;
                    c.V().ca_cpu()[m] = pres ? M.ps_cpu : 0u;
                    c.V().ca_ram()[m] = pres ? M.ps_ram : 0ull;
                }
                wave_sync();
                copied = true;
            }
            uint32_t nundo = 0;
            bool ok = true;
            for (uint32_t i = 0; i < k; i++) {
                const uint32_t p = uniform_u32(sorted[i]);
                const uint32_t rc = uniform_u32(c.V().pod(p).req_cpu);
                const uint64_t rr = uniform_u64(c.V().pod(p).req_ram);
                if (rc == 0 && rr == 0) {   // fits any other PS node; (0, 0) absent entries must not count
                    if (c.H().ps_node_count < 2) {
                        ok = false;
                        break;
                    }
                    continue;
                }
                const int32_t m = ca_first_fit(c, N, n, rc, rr);
                if (m < 0) {
                    ok = false;
                    break;
                }
                c.V().ca_cpu()[m] -= rc;
                c.V().ca_ram()[m] -= rr;
                if (nundo >= c.Ly().cap_undo) {
                    fail(c, K10S_ERR_CA_BUFFER);
                    return;
                }
                c.V().ca_undo()[2 * nundo] = (uint32_t)m;
                c.V().ca_undo()[2 * nundo + 1] = p;
                nundo++;
                wave_sync();
            }
            if (!ok) {
                for (uint32_t i = 0; i < nundo; i++) {  // *nodes = original
                    const uint32_t m = uniform_u32(c.V().ca_undo()[2 * i]), p = uniform_u32(c.V().ca_undo()[2 * i + 1]);
                    c.V().ca_cpu()[m] += c.V().pod(p).req_cpu;
                    c.V().ca_ram()[m] += c.V().pod(p).req_ram;
                    wave_sync();
                }
                return;
            }
        }
        if (nrem >= c.Ly().cap_act) {
            fail(c, K10S_ERR_CA_BUFFER);
            return;
        }
        c.V().ca_act()[nrem].up = 0;
        c.V().ca_act()[nrem].arg = n;
        nrem++;
    });
    if (c.H().error_code) return;
    for (uint32_t i = 0; i < nrem; i++) {
        uint32_t n = uniform_u32(c.V().ca_act()[i].arg);
        int32_t g = sc->def_ca_group[c.V().node(n).ps_def];
        if (g < 0) {
            fail(c, K10S_PANIC_CA_GROUP);
            return;
        }
        cag[2 * g] -= 1;
    }
    h->ca_n_act = nrem;
}

// ---- persistent storage (persistent_storage.rs:185-490) --------------------------------------
// The PS assignment set of a CA-origin node as an intrusive doubly-linked list (insertion order;
// the CA sorts a node's members by name when it needs them, kube_cluster_autoscaler.rs:271-277).
K10S_HD void ps_list_insert(Ctx& c, uint32_t n, uint32_t p) {
    int32_t* link = c.V().ps_link();
    const int32_t h = c.V().ps_head()[n];
    link[2 * p] = -1;
    link[2 * p + 1] = h;
    if (h >= 0) link[2 * h] = (int32_t)p;
    c.V().ps_head()[n] = (int32_t)p;
}
K10S_HD void ps_list_remove(Ctx& c, uint32_t n, uint32_t p) {
    int32_t* link = c.V().ps_link();
    const int32_t pr = link[2 * p], nx = link[2 * p + 1];
    if (pr >= 0) link[2 * pr + 1] = nx;
    else c.V().ps_head()[n] = nx;
    if (nx >= 0) link[2 * nx] = pr;
}

// The node line's storage fields, loaded in one batch.
struct PsNode {
    uint8_t flags;
    uint32_t cpu, epoch;
    uint64_t ram;
};
K10S_HD PsNode ps_node_load(Ctx& c, uint32_t n) {
    const NodeState& N = c.V().node(n);
    PsNode v;
    v.flags = N.flags;
    v.cpu = N.ps_cpu;
    v.epoch = N.ps_epoch;
    v.ram = N.ps_ram;
    return v;
}
// clean_up_pod (173-182) with the pod's fields loaded (n = ps_assigned) and node n's fields v.
K10S_HD void ps_clean_up_at(Ctx& c, uint32_t p, int32_t n, uint32_t rc, uint64_t rr, uint32_t pae, const PsNode& v) {
    if (n < 0) return;
    if (v.flags & NF_PS_PRESENT) {
        NodeState& N = c.V().node(n);
        N.ps_cpu = v.cpu + rc;
        N.ps_ram = v.ram + rr;
        if (pae == v.epoch) {
            c.V().pod(p).ps_aepoch = 0;
            if (v.flags & NF_CA_ORIGIN) ps_list_remove(c, (uint32_t)n, p);
        }
    }
}
K10S_HD void ps_clean_up(Ctx& c, uint32_t p) {  // 173-182
    PodState& P = c.V().pod(p);
    const int32_t n = P.ps_assigned;
    const uint32_t rc = P.req_cpu, pae = P.ps_aepoch;
    const uint64_t rr = P.req_ram;
    if (n < 0) return;
    ps_clean_up_at(c, p, n, rc, rr, pae, ps_node_load(c, (uint32_t)n));
}

K10S_WARM void on_ps(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    RepHdr* h = &c.H();
    const Params* pr = &c.P();
    switch (e.kind) {
    case K10S_EV_PS_CREATE_NODE_REQ: {
        uint32_t def = e.b, n = e.a;
        if (c.V().node(n).flags & NF_PS_PRESENT) {
            fail(c, K10S_PANIC_DUPLICATE_NODE);
            return;
        }
        // NF_CA_ORIGIN (and the assignment list behind it) only when the CA runs: its only reader
        const bool ca_origin = c.S().ca_enabled && c.S().def_ca_origin[def] != 0;
        c.V().node(n).flags = (uint8_t)((c.V().node(n).flags & ~NF_CA_ORIGIN) | NF_PS_PRESENT | (ca_origin ? NF_CA_ORIGIN : 0));
        c.V().node(n).ps_def = def;
        c.V().node(n).ps_cpu = c.S().def_cpu[def];
        c.V().node(n).ps_ram = c.S().def_ram[def];
        c.V().node(n).ps_epoch += 1;
        h->ps_node_count += 1;
        if (ca_origin) {  // a new, empty assignment set (persistent_storage.rs:70-84)
            c.V().ps_head()[n] = -1;
            bit_set(c.V().ca_live(), n);
        }
        emit(c, K10S_EV_AS_CREATE_NODE_RESP, pr->as_to_ps_network_delay, -1, n, 0, 0.0, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_PS_NODE_ADDED: {
        uint32_t n = e.a;
        if (!(c.V().node(n).flags & NF_PS_PRESENT)) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        emit(c, K10S_EV_S_ADD_NODE, pr->ps_to_sched_network_delay, -1, n, c.V().node(n).ps_cpu, u2f(c.V().node(n).ps_ram), FQ_PS_TO_SCHED);
        h->counters[K10S_C_PROCESSED_NODES] += 1;
        break;
    }
    case K10S_EV_PS_CREATE_POD_REQ: {
        uint32_t p = e.a;
        const uint8_t pf = c.V().pod(p).flags;
        if (pf & PF_IN_PS) {
            fail(c, K10S_PANIC_DUPLICATE_POD);
            return;
        }
        c.V().pod(p).flags = (uint8_t)(pf | PF_IN_PS);
        if (pf & PF_UNSCHED) h->unsched_missing -= 1;  // a re-created pod of the unscheduled cache
        c.V().pod(p).ps_assigned = -1;
        if (c.V().prec()) c.V().prec()[p].state = 1;
        emit(c, K10S_EV_S_POD_SCHEDULE_REQ, pr->ps_to_sched_network_delay, -1, p, 0, 0.0, FQ_PS_TO_SCHED);
        break;
    }
    case K10S_EV_PS_ASSIGN_REQ: {
        uint32_t p = e.a, n = e.b;
        PodState& P = c.V().pod(p);
        NodeState& N = c.V().node(n);
        const uint8_t pf = P.flags, nf = N.flags;  // one batch of loads (pod line, node line)
        const uint32_t rc = P.req_cpu, ncpu = N.ps_cpu, nep = N.ps_epoch;
        const uint64_t rr = P.req_ram, nram = N.ps_ram;
        if (!(pf & PF_IN_PS)) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        P.ps_assigned = (int32_t)n;
        if (pf & PF_UNSCHED) {
            P.flags = (uint8_t)(pf & ~PF_UNSCHED);
            h->unsched_cache_count -= 1;
            if (c.S().ca_enabled) bit_clear(c.V().ca_ubits(), p);
        }
        if (!(nf & NF_PS_PRESENT)) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        N.ps_cpu = ncpu - rc;
        N.ps_ram = nram - rr;
        P.ps_aepoch = nep;
        if (nf & NF_CA_ORIGIN) ps_list_insert(c, n, p);
        emit(c, K10S_EV_AS_ASSIGN_RESP, pr->as_to_ps_network_delay, -1, p, n, 0.0, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_PS_POD_NOT_SCHEDULED: {
        uint32_t p = e.a;
        if (!(c.V().pod(p).flags & PF_IN_PS)) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        if (!(c.V().pod(p).flags & PF_UNSCHED)) {
            c.V().pod(p).flags |= PF_UNSCHED;
            h->unsched_cache_count += 1;
            if (c.S().ca_enabled) bit_set(c.V().ca_ubits(), p);
        }
        break;
    }
    case K10S_EV_PS_POD_STARTED: {
        uint32_t p = e.a;
        // A pod leaves storage on its PodFinishedRunning or on a removal request.  Its
        // PodStartedRunning precedes its PodFinishedRunning here (both come through the api server's
        // ring to storage, started first: N_BIND emits the finish self-event at t + dur + d and the
        // start at t + d, and at dur = 0 the finish, handled first, re-emits after the start), so
        // while no removal request has dropped a pod (ps_rm_n == 0) the membership check cannot fail
        // and the pod line is not read.  That needs durations >= 0 (a negative one can land the
        // finish in storage before the start, persistent_storage.rs:313 then panics): the shortcut is
        // taken only in the default kernel copy (K10S_TIME_KEY_ID: every duration >= 0 by routing).
#if !K10S_DEVICE
        // the host check build verifies the invariant the shortcut relies on at every such event of
        // a scenario the default copy would run
        if (c.Ly().tnonneg && h->ps_rm_n == 0 && !(c.V().pod(p).flags & PF_IN_PS)) {
            fail(c, K10S_ERR_INVARIANT);
            return;
        }
#endif
        if ((!K10S_TIME_KEY_ID || h->ps_rm_n != 0) && !(c.V().pod(p).flags & PF_IN_PS)) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        if (c.V().prec()) c.V().prec()[p].t_running = e.x;
        break;
    }
    case K10S_EV_PS_POD_FINISHED: {
        uint32_t p = e.a;
        PodState& P = c.V().pod(p);
        // one batch of loads: the pod line, and the line of the node the pod ran on (e.b), which is
        // its storage assignment unless the assignment changed meanwhile (then reloaded below)
        const uint32_t hn = e.b < c.S().n_nodes ? e.b : 0u;
        const PsNode hv = ps_node_load(c, hn);
        const uint8_t pf = P.flags, sflags = c.S().pod_flags[p];
        const double dur = P.dur;
        const int32_t pn = P.ps_assigned;
        const uint32_t prc = P.req_cpu, pae = P.ps_aepoch;
        const uint64_t prr = P.req_ram;
        if (pf & PF_IN_PS) {
            P.flags = (uint8_t)(pf & ~PF_IN_PS);
            if (pf & PF_UNSCHED) h->unsched_missing += 1;
            if (pn >= 0) ps_clean_up_at(c, p, pn, prc, prr, pae, (uint32_t)pn == hn ? hv : ps_node_load(c, (uint32_t)pn));
            if (!(sflags & POD_HAS_DUR)) {
                fail(c, K10S_PANIC_MISSING_POD);
                return;
            }
            est_add(h->est[K10S_EST_POD_DURATION], dur);
            if (c.V().prec()) {
                c.V().prec()[p].t_finished = e.x;
                c.V().prec()[p].state = 2;
            }
        }
        emit(c, K10S_EV_S_POD_FINISHED, pr->ps_to_sched_network_delay, -1, p, e.b, e.x, FQ_PS_TO_SCHED);
        break;
    }
    case K10S_EV_PS_REMOVE_NODE_REQ: {
        uint32_t n = e.a;
        if (!(c.V().node(n).flags & NF_PS_PRESENT)) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        if (c.V().node(n).flags & NF_CA_ORIGIN) bit_clear(c.V().ca_live(), n);
        c.V().node(n).flags &= (uint8_t)~(NF_PS_PRESENT | NF_CA_ORIGIN);
        h->ps_node_count -= 1;
        emit(c, K10S_EV_AS_REMOVE_NODE_RESP, pr->as_to_ps_network_delay, -1, n, 0, 0.0, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_PS_NODE_REMOVED:
        emit(c, K10S_EV_S_REMOVE_NODE, pr->ps_to_sched_network_delay, -1, e.a, 0, 0.0, FQ_PS_TO_SCHED);
        break;
    case K10S_EV_PS_REMOVE_POD_REQ: {
        uint32_t p = e.a;
        if (!(c.V().pod(p).flags & PF_IN_PS)) {
            emit(c, K10S_EV_AS_REMOVE_POD_RESP, pr->as_to_ps_network_delay, -1, p, 0, 0.0, FQ_AS_TO_PS);
            return;
        }
        if (c.V().pod(p).flags & PF_UNSCHED) h->unsched_missing += 1;
        c.V().pod(p).flags &= (uint8_t)~PF_IN_PS;
        h->ps_rm_n += 1;
        if (c.V().prec()) {
            c.V().prec()[p].t_removed = e.time;
            c.V().prec()[p].state = 3;
        }
        int32_t n = c.V().pod(p).ps_assigned;
        uint32_t flag = 0;
        if (n >= 0) {
            ps_clean_up(c, p);
            flag = 1;
        } else {
            emit(c, K10S_EV_S_REMOVE_POD, pr->ps_to_sched_network_delay, -1, p, 0, 0.0, FQ_PS_TO_SCHED);
        }
        emit(c, K10S_EV_AS_REMOVE_POD_RESP, pr->as_to_ps_network_delay, -1, p, flag ? (uint32_t)n : 0u, u2f(flag), FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_PS_POD_REMOVED:
        if (e.b) emit(c, K10S_EV_S_REMOVE_POD, pr->ps_to_sched_network_delay, -1, e.a, 0, 0.0, FQ_PS_TO_SCHED);
        break;
    default:
        break;
    }
}

// Storage's ClusterAutoscalerRequest (persistent_storage.rs:381-412): the CA decision.  Its own
// out-of-line handler, not a case of on_ps: the registers ca_decide clobbers then do not count against
// on_ps, whose call the event loop makes four times per pod (with the decision inside, the loop saved
// and restored 20 SGPRs around every on_ps call: 40 VALU lane moves).
K10S_COLD void on_ps_ca(Ctx& c, K10S_EVARG) {
    (void)ep;
    ca_decide(c);
    emit(c, K10S_EV_AS_CA_RESP, c.P().as_to_ps_network_delay, -1, 0, 0, 0.0, FQ_AS_TO_PS);
}

// The api server's removal set (names with a removal in flight, api_server.rs:343, 285-305) as a
// uid bitset with its population count in the header.
K10S_HD void pend_rm_set(Ctx& c, uint32_t uid) {
    if (!bit_test(c.V().pend_rm(), uid)) {
        bit_set(c.V().pend_rm(), uid);
        c.H().pend_rm_n += 1;
    }
}
K10S_HD void pend_rm_clear(Ctx& c, uint32_t uid) {
    if (bit_test(c.V().pend_rm(), uid)) {
        bit_clear(c.V().pend_rm(), uid);
        c.H().pend_rm_n -= 1;
    }
}

// ---- the finish relay handled with the finish (round 5) -------------------------------------------
// A node component's PodFinishedRunning self-event at time T emits the api server's
// PodFinishedRunning with emit_now (node_component.rs:227-245): the relay gets time T and the next id,
// so it is the very next event exactly when no other pending event has a time <= T (one at T has a
// smaller id and goes first; no later-emitted event can precede it).  Then the finish handler handles
// the relay itself (api_server.rs:247-276: counters, pods left, a PS_POD_FINISHED after as_to_ps)
// with the id the relay would have had, logged and counted as an event, instead of a round through
// the FIFO of delay 0 and the event loop.  Pending events: the other sources' heads (the source
// list's second entry is the smallest) and the heap below its root, which is the finish itself (the
// root's children hold the heap's second-smallest entry: one LDS read of the top level, a canceled
// finish counting like a live one).  Not fused: a budgeted launch (the loop may stop between the
// two), a launch the termination rule would end before the relay (pods_left <= 0 at a multiple of
// 1,000 s), an id overflow.
#ifndef K10S_FUSE_FINISH
#define K10S_FUSE_FINISH 1
#endif
// api_server.rs:247-276 (PodFinishedRunning): the serial handler and the fused relay
K10S_HD void as_pod_finished(Ctx& c, uint32_t a, uint32_t b, double x) {
    RepHdr* h = &c.H();
    h->counters[K10S_C_TERMINATED_PODS] += 1;
    pods_left_dec(*h);
    h->counters[K10S_C_PODS_SUCCEEDED] += 1;
    h->g_cur_pods -= 1;  // api_server.rs:262-265
    emit(c, K10S_EV_PS_POD_FINISHED, c.P().as_to_ps_network_delay, -1, a, b, x, FQ_AS_TO_PS);
}
// Is the relay of a finish at time T (the heap root) the next event?
K10S_HD bool finish_relay_next(Ctx& c, double T) {
    if (!K10S_FUSE_FINISH) return false;
    RepHdr& H = c.H();
    const uint32_t fl = uniform_u32(H.run_flags);
    if (!(fl & 1u)) return false;
    if (!(fl & 2u) && (int64_t)uniform_u64((uint64_t)H.pods_left) <= 0 && is_multiple_of_1000(T)) return false;
    if (uniform_u32(H.next_seq) >= 0xFFFFFFFEu) return false;
    if (uniform_u32(H.sl[0].src) != (uint32_t)SRC_HEAP) return false;
    const int64_t kT = total_key(T);
    if (uniform_u32(H.sl_n) > 1 && (int64_t)uniform_u64((uint64_t)H.sl[1].key) <= kT) return false;
    const uint32_t n = uniform_u32(H.heap_size);
    static_assert(K10S_HEAP_TOP >= 1 + K10S_HEAP_D, "the root's children are in the LDS top level");
#if K10S_DEVICE
    const uint32_t i = 1u + (uint32_t)lane_id();
    const bool early = i < n && i <= (uint32_t)K10S_HEAP_D && total_key(H.heap_lds[i < K10S_HEAP_TOP ? i : 0].time) <= kT;
    return __ballot(early) == 0;
#else
    for (uint32_t i = 1; i < n && i <= (uint32_t)K10S_HEAP_D; i++)
        if (total_key(H.heap_lds[i].time) <= kT) return false;
    return true;
#endif
}
// The fused relay: the id, the log entry and the event count the loop would give it, then its handler.
K10S_HD void as_pod_finished_fused(Ctx& c, uint32_t a, uint32_t b, double x, double T) {
    RepHdr& H = c.H();
    const uint32_t seq = uniform_u32(H.next_seq);
    H.next_seq = seq + 1u;
    const uint32_t cap_log = c.Ly().cap_log;
    if (cap_log) {
        const uint32_t k = uniform_u32(H.log_n);
        if (k < cap_log) {
            k10s_log_entry le;
            le.time = T;
            le.seq = seq;
            le.kind = (uint16_t)K10S_EV_AS_POD_FINISHED;
            le.slot = -1;
            le.pod = (int32_t)a;
            le.node = (int32_t)b;
            c.V().log()[k] = le;
            H.log_n = k + 1u;
        } else {
            H.flags |= 1u;
        }
    }
    H.counters[K10S_C_EVENTS] += 1;
#if K10S_PROF
    H.prof[K10S_PROF_KIND0 + K10S_EV_NUM_KINDS + K10S_EV_AS_POD_FINISHED] += 1;
#endif
    K10S_HSTAT(HS_FUSED_FINISH);
    as_pod_finished(c, a, b, x);
}

// ---- api server (api_server.rs:127-457) --------------------------------------------------------
K10S_WARM void on_api_server(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    RepHdr* h = &c.H();
    const Params* pr = &c.P();
    const Scenario* sc = &c.S();
    switch (e.kind) {
    case K10S_EV_AS_CREATE_NODE_REQ: {
        uint32_t def = e.b;
        uint32_t n = sc->def_node[def];
        h->g_cur_nodes += 1;  // api_server.rs:133-137
        c.V().node(n).pend_def = (int32_t)def;
        emit(c, K10S_EV_PS_CREATE_NODE_REQ, pr->as_to_ps_network_delay, -1, n, def, 0.0, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_AS_CREATE_NODE_RESP: {  // handle_create_node (96-115)
        uint32_t n = e.a;
        int32_t def = c.V().node(n).pend_def;
        if (def < 0) {
            fail(c, K10S_PANIC_MISSING_PENDING);
            return;
        }
        c.V().node(n).pend_def = -1;
        if (h->pool_count == 0) {
            fail(c, K10S_PANIC_POOL_EXHAUSTED);
            return;
        }
        uint32_t slot = c.V().pool_ring()[h->pool_head];
        h->pool_head = (h->pool_head + 1) % sc->n_slots;
        h->pool_count -= 1;
        c.V().slot(slot).node = (int32_t)n;
        c.V().slot(slot).def = (uint32_t)def;
        if (c.V().node(n).as_slot >= 0) {
            fail(c, K10S_PANIC_DUPLICATE_NODE);
            return;
        }
        c.V().node(n).as_slot = (int32_t)slot;
        h->as_node_count += 1;
        if (c.Ly().cap_gauge) {  // the component's node: allocatable = capacity (api_server.rs:133)
            c.V().g_cpu()[slot] = sc->def_cpu[def];
            c.V().g_ram()[slot] = sc->def_ram[def];
        }
        emit(c, K10S_EV_PS_NODE_ADDED, pr->as_to_ps_network_delay, -1, n, 0, e.time, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_AS_CREATE_POD_REQ:
        h->g_cur_pods += 1;  // api_server.rs:151-155
        emit(c, K10S_EV_PS_CREATE_POD_REQ, pr->as_to_ps_network_delay, -1, e.a, 0, 0.0, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_ASSIGN_REQ: {
        uint32_t n = e.b;
        const int32_t as_slot = c.V().node(n).as_slot;  // loaded with the removal bit, not after it
        const bool pending = h->pend_rm_n != 0 && bit_test(c.V().pend_rm(), sc->node_uid[n]);
        if (pending || as_slot < 0) return;
        emit(c, K10S_EV_PS_ASSIGN_REQ, pr->as_to_ps_network_delay, -1, e.a, n, e.x, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_AS_ASSIGN_RESP: {
        uint32_t n = e.b;
        int32_t slot = c.V().node(n).as_slot;
        if (slot < 0) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        emit(c, K10S_EV_N_BIND, pr->as_to_node_network_delay, slot, e.a, n, 0.0, FQ_AS_TO_NODE);
        break;
    }
    case K10S_EV_AS_POD_NOT_SCHEDULED:
        emit(c, K10S_EV_PS_POD_NOT_SCHEDULED, pr->as_to_ps_network_delay, -1, e.a, 0, e.x, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_POD_STARTED:
        emit(c, K10S_EV_PS_POD_STARTED, pr->as_to_ps_network_delay, -1, e.a, 0, e.x, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_POD_FINISHED:
        as_pod_finished(c, e.a, e.b, e.x);
        break;
    case K10S_EV_AS_REMOVE_NODE_REQ:
        pend_rm_set(c, sc->node_uid[e.a]);
        emit(c, K10S_EV_PS_REMOVE_NODE_REQ, pr->as_to_ps_network_delay, -1, e.a, 0, 0.0, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_REMOVE_NODE_RESP: {
        int32_t slot = c.V().node(e.a).as_slot;
        if (slot < 0) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        emit(c, K10S_EV_N_REMOVE_NODE, pr->as_to_node_network_delay, slot, e.a, 0, 0.0, FQ_AS_TO_NODE);
        break;
    }
    case K10S_EV_AS_NODE_REMOVED: {
        uint32_t n = e.a;
        int32_t slot = c.V().node(n).as_slot;
        if (slot < 0) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        c.V().node(n).as_slot = -1;
        h->as_node_count -= 1;
        h->g_cur_nodes -= 1;  // api_server.rs:301-304
        // reclaim_component (node_component_pool.rs:68-77)
        c.V().slot(slot).node = -1;
        c.V().slot(slot).removed = 0;
        c.V().slot(slot).rtime = 0.0;
        c.V().slot(slot).gen += 1;
        c.V().slot(slot).running = 0;
        uint32_t tail = (h->pool_head + h->pool_count) % sc->n_slots;
        c.V().pool_ring()[tail] = (uint32_t)slot;
        h->pool_count += 1;
        pend_rm_clear(c, sc->node_uid[n]);
        emit(c, K10S_EV_PS_NODE_REMOVED, pr->as_to_ps_network_delay, -1, n, 0, e.x, FQ_AS_TO_PS);
        break;
    }
    case K10S_EV_AS_CA_REQ:
        emit(c, K10S_EV_PS_CA_REQ, pr->as_to_ps_network_delay, -1, 0, 0, 0.0, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_CA_RESP:
        emit(c, K10S_EV_CA_RESP, pr->as_to_ca_network_delay, -1, 0, 0, 0.0, FQ_AS_TO_CA);
        break;
    case K10S_EV_AS_REMOVE_POD_REQ:
        pend_rm_set(c, sc->pod_uid[e.a]);  // quirk (api_server.rs:343): the NODE removal set
        emit(c, K10S_EV_PS_REMOVE_POD_REQ, pr->as_to_ps_network_delay, -1, e.a, 0, 0.0, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_REMOVE_POD_RESP: {
        if (f2u(e.x) != 0) {
            int32_t slot = c.V().node(e.b).as_slot;
            if (slot < 0) {
                fail(c, K10S_PANIC_MISSING_NODE);
                return;
            }
            emit(c, K10S_EV_N_REMOVE_POD, pr->as_to_node_network_delay, slot, e.a, e.b, 0.0, FQ_AS_TO_NODE);
        }
        break;
    }
    case K10S_EV_AS_POD_REMOVED:
        if (e.b) {
            h->counters[K10S_C_TERMINATED_PODS] += 1;
            pods_left_dec(*h);
            h->counters[K10S_C_PODS_REMOVED] += 1;
            h->g_cur_pods -= 1;  // api_server.rs:388-391
        }
        emit(c, K10S_EV_PS_POD_REMOVED, pr->as_to_ps_network_delay, -1, e.a, e.b, e.x, FQ_AS_TO_PS);
        break;
    case K10S_EV_AS_CREATE_GROUP_REQ: {
        uint32_t g = e.a;
        if (sc->g_flags[g] & GF_TMPL_HAS_DUR) {
            fail(c, K10S_PANIC_GROUP_DURATION);
            return;
        }
        GroupState& gs = c.V().grp()[g];
        gs.creation_time = e.time;
        gs.cpu_last_start = e.time;
        gs.ram_last_start = e.time;
        gs.cpu_idx = 0;
        gs.ram_idx = 0;
        gs.created_at_as = 1;
        uint32_t init = sc->g_initial[g];
        if (init > sc->group_bound) {
            fail(c, K10S_ERR_NAME_BOUND);
            return;
        }
        h->g_cur_pods += init;  // api_server.rs:442-446
        for (uint32_t k = 0; k < init && !c.H().error_code; k++)
            emit(c, K10S_EV_PS_CREATE_POD_REQ, pr->as_to_ps_network_delay, -1, sc->g_pod[g * sc->group_bound + k], 0, 0.0, FQ_AS_TO_PS);
        if (sc->hpa_enabled) emit(c, K10S_EV_HPA_REGISTER_GROUP, pr->as_to_hpa_network_delay, -1, g, 0, e.time, FQ_AS_TO_HPA);
        break;
    }
    default:
        break;
    }
}

// ---- node components (node_component.rs:178-335) ------------------------------------------------
K10S_WARM void on_node(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    const Params* pr = &c.P();
    int32_t slot = e.slot;
    switch (e.kind) {
    case K10S_EV_N_BIND: {
        uint32_t p = e.a, n = e.b;
        // one batch of loads: the component's slot line, the pod line and the pod's scenario flags
        SlotState& SL = c.V().slot(slot);
        PodState& P = c.V().pod(p);
        const uint32_t removed = SL.removed;
        const int32_t snode = SL.node, srun = SL.running;
        const int32_t prs = P.run_slot;
        const double dur = P.dur;
        const uint8_t sflags = c.S().pod_flags[p];
        const int32_t g = c.S().pod_group[p];
        if (removed) {
            fail(c, K10S_PANIC_BIND_REMOVED_NODE);
            return;
        }
        if (snode != (int32_t)n) {
            fail(c, K10S_PANIC_BIND_REMOVED_NODE);
            return;
        }
        if (prs >= 0) {  // a second concurrent bind of one pod: not modelled
            fail(c, K10S_PANIC_BIND_REMOVED_NODE);
            return;
        }
        uint32_t fseq = 0;
        if (sflags & POD_HAS_DUR)  // simulate_pod_runtime (114-175)
            fseq = emit(c, K10S_EV_N_POD_FINISHED, dur + pr->as_to_node_network_delay, slot, p, n, e.time + dur);
        SL.running = srun + 1;   // the count loaded above (emit touches only the event queue)
        P.run_slot = slot;
        P.finish_seq = fseq;
        if (c.Ly().cap_gauge) {  // allocate_pod_requests (node_component.rs:83-86, called at 164)
            c.V().g_cpu()[slot] -= P.req_cpu;
            c.V().g_ram()[slot] -= P.req_ram;
        }
        if (g >= 0) c.V().grp()[g].running += 1;
        emit(c, K10S_EV_AS_POD_STARTED, pr->as_to_node_network_delay, -1, p, 0, e.time, FQ_AS_TO_NODE);
        break;
    }
    case K10S_EV_N_POD_FINISHED: {
        uint32_t p = e.a;
        // one batch of loads: the pod line, the component's count (the event names the component)
        // and the pod's group (scenario)
        const int32_t rs = c.V().pod(p).run_slot;
        const uint32_t fs = c.V().pod(p).finish_seq;
        const int32_t srun = c.V().slot(slot).running;
        const int32_t g = c.S().pod_group[p];
        if (rs != slot) {
            fail(c, K10S_PANIC_MISSING_POD);
            return;
        }
        run_remove_at(c, p, slot, fs, srun, g);
        if (finish_relay_next(c, e.time)) as_pod_finished_fused(c, p, e.b, e.x, e.time);
        else emit(c, K10S_EV_AS_POD_FINISHED, 0.0, -1, p, e.b, e.x, FQ_NOW);  // emit_now
        break;
    }
    case K10S_EV_N_REMOVE_NODE: {
        uint32_t n = e.a;
        if (c.V().slot(slot).node != (int32_t)n) {
            fail(c, K10S_PANIC_REMOVE_OTHER_NODE);
            return;
        }
        // cancel_all_running_pods (95-112): the pods whose run_slot is this component, in index order
        // (the per-pod work is order-independent)
        const uint32_t gen = c.V().slot(slot).gen;
        if (c.V().slot(slot).running > 0)
            for_each_pod_in_order(
                c, [&](uint32_t p) { return c.V().pod(p).run_slot == slot; },
                [&](uint32_t p) {
                    c.V().pod(p).cancel_slot = slot;
                    c.V().pod(p).cancel_gen = gen;
                    run_remove(c, p);
                });
        emit(c, K10S_EV_AS_NODE_REMOVED, pr->as_to_node_network_delay, -1, n, 0, e.time, FQ_AS_TO_NODE);
        c.V().slot(slot).removed = 1;
        c.V().slot(slot).rtime = e.time;
        break;
    }
    case K10S_EV_N_REMOVE_POD: {
        uint32_t p = e.a;
        if (c.V().slot(slot).node < 0) {
            fail(c, K10S_PANIC_MISSING_NODE);
            return;
        }
        if (c.V().pod(p).run_slot == slot) {
            run_remove(c, p);
            emit(c, K10S_EV_AS_POD_REMOVED, pr->as_to_node_network_delay, -1, p, 1, e.time, FQ_AS_TO_NODE);
        } else if (c.V().pod(p).cancel_slot == slot && c.V().pod(p).cancel_gen == c.V().slot(slot).gen) {
            emit(c, K10S_EV_AS_POD_REMOVED, pr->as_to_node_network_delay, -1, p, 1, c.V().slot(slot).rtime, FQ_AS_TO_NODE);
        } else {
            emit(c, K10S_EV_AS_POD_REMOVED, pr->as_to_node_network_delay, -1, p, 0, 0.0, FQ_AS_TO_NODE);
        }
        break;
    }
    default:
        break;
    }
}

// ---- cluster autoscaler proxy (cluster_autoscaler.rs:230-334) --------------------------------
K10S_COLD void on_ca(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    RepHdr* h = &c.H();
    const Params* pr = &c.P();
    if (e.kind == K10S_EV_CA_TICK) {
        h->ca_last_cycle_time = e.time;
        emit(c, K10S_EV_AS_CA_REQ, pr->as_to_ca_network_delay, -1, 0, 0, 0.0, FQ_AS_TO_CA);
        return;
    }
    for (uint32_t i = 0; i < h->ca_n_act && !c.H().error_code; i++) {
        CAAct a = c.V().ca_act()[i];
        if (a.up) {
            emit(c, K10S_EV_AS_CREATE_NODE_REQ, pr->as_to_ca_network_delay, -1, c.S().def_node[a.arg], a.arg, 0.0, FQ_AS_TO_CA);
            h->counters[K10S_C_TOTAL_SCALED_UP_NODES] += 1;
        } else {
            emit(c, K10S_EV_AS_REMOVE_NODE_REQ, pr->as_to_ca_network_delay, -1, a.arg, 0, 0.0, FQ_AS_TO_CA);
            h->counters[K10S_C_TOTAL_SCALED_DOWN_NODES] += 1;
        }
    }
    h->ca_n_act = 0;
    double delay = pr->ca_scan_interval;
    if (e.time - h->ca_last_cycle_time > pr->ca_scan_interval) delay = 0.0;
    emit0(c, K10S_EV_CA_TICK, delay);
}

// ---- HPA (horizontal_pod_autoscaler.rs:146-257, kube_horizontal_pod_autoscaler.rs:54-216) ----
// Groups are visited in name order (the reference iterates a HashMap: A.5).
K10S_HD uint32_t hpa_desired_by_metric(uint32_t cur, double value, double target, double tol) {
    double ratio = value / target;
    if (__builtin_fabs(ratio - 1.0) <= tol) return cur;
    uint64_t d = f64_as_u64(__builtin_ceil((double)cur * ratio));
    return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

K10S_COLD void on_hpa(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    RepHdr* h = &c.H();
    const Scenario* sc = &c.S();
    const uint32_t B = sc->group_bound;
    const uint32_t words = c.Ly().words_group;
    if (e.kind == K10S_EV_HPA_REGISTER_GROUP) {
        uint32_t g = e.a;
        GroupState& gs = c.V().grp()[g];
        gs.registered = 1;
        uint64_t* bits = c.V().grp_bits() + (uint64_t)g * words;
        for (uint32_t i = 0; i < words; i++) bits[i] = 0;
        uint32_t init = sc->g_initial[g];
        for (uint32_t k = 0; k < init; k++) bit_set(bits, sc->g_pos[g * B + k]);
        gs.created_count = init;
        gs.total_created = init;
        return;
    }
    for (uint32_t g = 0; g < sc->n_groups && !c.H().error_code; g++) {
        GroupState& gs = c.V().grp()[g];
        if (!gs.has_metric) continue;
        if (!gs.registered) {
            fail(c, K10S_PANIC_HPA_UNREGISTERED);
            return;
        }
        uint8_t gf = sc->g_flags[g];
        uint32_t cur = gs.created_count;
        const double tol = c.P().hpa_target_threshold_tolerance;
        uint32_t dc = (gf & GF_HAS_TCPU) ? hpa_desired_by_metric(cur, gs.util_cpu, sc->g_tcpu[g], tol) : 0;
        uint32_t dr = (gf & GF_HAS_TRAM) ? hpa_desired_by_metric(cur, gs.util_ram, sc->g_tram[g], tol) : 0;
        uint32_t mx = sc->g_max[g];
        uint32_t desired;
        if ((gf & GF_HAS_TCPU) && (gf & GF_HAS_TRAM)) desired = (dc > dr ? dc : dr) < mx ? (dc > dr ? dc : dr) : mx;
        else if (gf & GF_HAS_TCPU) desired = dc < mx ? dc : mx;
        else if (gf & GF_HAS_TRAM) desired = dr < mx ? dr : mx;
        else desired = cur;
        uint64_t* bits = c.V().grp_bits() + (uint64_t)g * words;
        if (cur < desired) {
            for (uint32_t i = 0; i < desired - cur && !c.H().error_code; i++) {
                uint32_t k = gs.total_created;
                if (k >= B) {
                    fail(c, K10S_ERR_NAME_BOUND);
                    return;
                }
                bit_set(bits, sc->g_pos[g * B + k]);
                gs.created_count += 1;
                gs.total_created += 1;
                emit(c, K10S_EV_AS_CREATE_POD_REQ, c.P().as_to_ca_network_delay, -1, sc->g_pod[g * B + k], 0, 0.0, FQ_AS_TO_CA);
                h->counters[K10S_C_TOTAL_SCALED_UP_PODS] += 1;
            }
        } else if (cur > desired) {
            for (uint32_t i = 0; i < cur - desired && !c.H().error_code; i++) {
                uint32_t j = 0;  // created_pods.pop_first(): smallest name
                for (uint32_t w = 0; w < words; w++) {
                    if (bits[w]) {
                        j = w * 64 + (uint32_t)__builtin_ctzll(bits[w]);
                        break;
                    }
                }
                bit_clear(bits, j);
                gs.created_count -= 1;
                uint32_t k = sc->g_sorted_k[g * B + j];
                emit(c, K10S_EV_AS_REMOVE_POD_REQ, c.P().as_to_ca_network_delay, -1, sc->g_pod[g * B + k], 0, 0.0, FQ_AS_TO_CA);
                h->counters[K10S_C_TOTAL_SCALED_DOWN_PODS] += 1;
            }
        }
    }
    emit0(c, K10S_EV_HPA_TICK, c.P().hpa_scan_interval);
}

// ---- metrics collector (collector.rs:263-337, 410-431) -----------------------------------------
K10S_HD double usage_poll(const Scenario* sc, uint8_t kind, double usage, uint32_t uoff, uint32_t ucnt, double& last_start,
                          uint32_t& idx, double t, uint32_t count) {
    if (kind == MODEL_NONE) return 0.0;
    if (kind == MODEL_CONSTANT) return usage;
    // PodGroupResourceUsageModel::current_usage (pod_group.rs:167-201)
    while (last_start + sc->unit_dur[uoff + idx] <= t) {
        last_start += sc->unit_dur[uoff + idx];
        idx = (idx + 1) % ucnt;
    }
    return fmin_rs(1.0, sc->unit_load[uoff + idx] / (double)count);
}

// ---- gauge recorder (collector.rs:352-407), opt-in (k10s_capacities.gauge_log) ------------------
#if K10S_DEVICE
K10S_D double lane_f64(double v, int l) {
    const uint64_t b = f2u(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return u2f((uint64_t)lo | ((uint64_t)hi << 32));
}
K10S_D uint64_t wave_sum_u64_cold(uint64_t v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor((unsigned long long)v, o);
    return v;
}
#endif
// collect_utilizations + record_gauge_metrics: one row per 5-s tick.  The lanes load 64 consecutive
// node indices at a time; the f64 node averages are then summed serially over the created nodes in
// name order (ascending index), the integer cluster sums in any order (exact).
K10S_COLD void gauge_record(Ctx& c, double t) {
    if (!K10S_FULL_WAVE(XG_GAUGE)) return;
    RepHdr* h = &c.H();
    if (h->gauge_n >= c.Ly().cap_gauge) {
        h->flags |= 4u;
        return;
    }
    const Scenario* sc = &c.S();
    const uint32_t N = sc->n_nodes;
    double navg_c = 0.0, navg_r = 0.0;
    uint64_t rq_c = 0, rq_r = 0, cap_c = 0, cap_r = 0, cnt = 0;
    for (uint32_t base = 0; base < N; base += K10S_LANES) {
        const uint32_t n = base + (uint32_t)lane_id();
        const int32_t slot = n < N ? c.V().node(n).as_slot : -1;
        double fc = 0.0, fr = 0.0;
        if (slot >= 0) {
            const uint32_t def = c.V().slot(slot).def;
            const uint64_t cc = sc->def_cpu[def], cr = sc->def_ram[def];
            const uint64_t qc = cc - (uint64_t)c.V().g_cpu()[slot], qr = cr - c.V().g_ram()[slot];
            fc = (double)qc / (double)cc;
            fr = (double)qr / (double)cr;
            rq_c += qc;
            rq_r += qr;
            cap_c += cc;
            cap_r += cr;
        }
#if K10S_DEVICE
        uint64_t m = __ballot(slot >= 0);
        cnt += (uint64_t)__popcll(m);
        while (m) {
            const int l = (int)uniform_u32((uint32_t)__builtin_ctzll(m));
            m &= m - 1;
            navg_c += lane_f64(fc, l);
            navg_r += lane_f64(fr, l);
        }
#else
        if (slot >= 0) {
            cnt += 1;
            navg_c += fc;
            navg_r += fr;
        }
#endif
    }
#if K10S_DEVICE
    rq_c = wave_sum_u64_cold(rq_c);
    rq_r = wave_sum_u64_cold(rq_r);
    cap_c = wave_sum_u64_cold(cap_c);
    cap_r = wave_sum_u64_cold(cap_r);
#endif
    k10s_gauge_row row;
    row.time = t;
    row.current_nodes = h->g_cur_nodes;
    row.current_pods = h->g_cur_pods;
    row.pods_in_scheduling_queues = h->g_pods_q;
    row.node_average_cpu_utilization = navg_c / (double)cnt;
    row.node_average_ram_utilization = navg_r / (double)cnt;
    row.cluster_total_cpu_utilization = (double)rq_c / (double)cap_c;
    row.cluster_total_ram_utilization = (double)rq_r / (double)cap_r;
    c.V().gauge()[h->gauge_n] = row;
    h->gauge_n += 1;
}

K10S_COLD void on_metrics(Ctx& c, K10S_EVARG) {
    K10S_EV_PROLOGUE;
    if (e.kind == K10S_EV_M_GAUGE_TICK) {  // CSV gauge record: no simulation state (collector.rs:392-407)
        if (c.Ly().cap_gauge) gauge_record(c, e.time);
        emit0(c, K10S_EV_M_GAUGE_TICK, 5.0);
        return;
    }
    const Scenario* sc = &c.S();
    for (uint32_t g = 0; g < sc->n_groups; g++) {
        GroupState& gs = c.V().grp()[g];
        gs.has_metric = gs.running > 0;
        if (!gs.has_metric) continue;
        // every pod of the group reports the same value (same model, creation time and count), so the
        // Mean estimator over them is exactly that value
        gs.util_cpu = usage_poll(sc, sc->g_cpu_kind[g], sc->g_cpu_usage[g], sc->g_cpu_uoff[g], sc->g_cpu_ucnt[g],
                                 gs.cpu_last_start, gs.cpu_idx, e.time, gs.running);
        gs.util_ram = usage_poll(sc, sc->g_ram_kind[g], sc->g_ram_usage[g], sc->g_ram_uoff[g], sc->g_ram_ucnt[g],
                                 gs.ram_last_start, gs.ram_idx, e.time, gs.running);
    }
    emit0(c, K10S_EV_M_POD_METRICS_TICK, 60.0);
}

// (Round 2 inlined the api server's forwarding cases here, K10S_FAST_DISPATCH: VGPR spills 20 -> 77,
// -3 % at C3, profiles/r02_v14_fast_dispatch_ab.json; not kept.)
// The kinds that come in runs (run_batch) go through their own out-of-line entry: it tries the run
// and otherwise calls the kind's handler.  The handlers themselves stay leaf functions (a call inside
// on_api_server / on_ps made them save their return address and a VGPR to scratch on every event),
// and the event loop pays one scalar mask test per event.
#define K10S_RUN_KINDS ((1ull << K10S_EV_AS_CREATE_POD_REQ) | (1ull << K10S_EV_PS_CREATE_POD_REQ) |      \
                        (1ull << K10S_EV_S_POD_SCHEDULE_REQ) | (1ull << K10S_EV_AS_CREATE_NODE_REQ) |    \
                        (1ull << K10S_EV_PS_CREATE_NODE_REQ) | (1ull << K10S_EV_AS_CREATE_NODE_RESP) |   \
                        (1ull << K10S_EV_PS_NODE_ADDED) | (1ull << K10S_EV_S_ADD_NODE))
#ifndef K10S_WINDOWS
#define K10S_WINDOWS 1
#endif
#ifndef K10S_WIN_NOTSCHED
#define K10S_WIN_NOTSCHED 1   // the failed attempts' relays in windows (A/B knob)
#endif
#define K10S_WIN_KINDS ((1ull << K10S_EV_AS_ASSIGN_REQ) | (1ull << K10S_EV_PS_ASSIGN_REQ) |                 \
                        (1ull << K10S_EV_AS_ASSIGN_RESP) | (1ull << K10S_EV_N_BIND) |                       \
                        (1ull << K10S_EV_AS_POD_STARTED) | (1ull << K10S_EV_PS_POD_STARTED) |               \
                        (K10S_WIN_NOTSCHED ? (1ull << K10S_EV_AS_POD_NOT_SCHEDULED) |                        \
                                                 (1ull << K10S_EV_PS_POD_NOT_SCHEDULED) : 0ull))
#define K10S_BATCH_KINDS (K10S_RUN_KINDS | (K10S_WINDOWS ? K10S_WIN_KINDS : 0ull))
// The scheduler's run kinds for on_run_kind's fallback: not on_scheduler itself, whose scheduling
// cycle (64 VGPRs) would make every call of on_run_kind clobber the event loop's live VGPRs (six
// 64-bit values spilled to scratch and reloaded around each call).
K10S_HD void on_scheduler_run_kind(Ctx& c, EvRef ep, uint32_t k) {
    HeapEv e = *ep;
    uniform_event(e);
    if (k == K10S_EV_S_ADD_NODE) s_add_node(c, e);
    else s_pod_schedule_req(c, e);
}
static_assert((K10S_BATCH_KINDS & (((1ull << (K10S_EV_S_REMOVE_POD + 1)) - 1ull) & ~((1ull << K10S_EV_S_RUN_CYCLE) - 1ull))) ==
                  ((1ull << K10S_EV_S_POD_SCHEDULE_REQ) | (1ull << K10S_EV_S_ADD_NODE)),
              "on_scheduler_run_kind handles every scheduler kind a batch entry can fall back to");
K10S_WARM void on_run_kind(Ctx& c, EvRef ep, uint32_t k) {
    k = uniform_u32(k);
    if ((K10S_RUN_KINDS >> k) & 1ull) {
        if (K10S_RUN_CALL(c, k)) return;
    } else {
        if (uniform_u32(win_batch(c)) != 0u) return;
    }
    if (k <= K10S_EV_AS_CREATE_GROUP_REQ) {
        on_api_server(c, ep);
    } else if (k <= K10S_EV_PS_POD_REMOVED) {
        on_ps(c, ep);
    } else if (k <= K10S_EV_S_REMOVE_POD) {
        on_scheduler_run_kind(c, ep, k);   // (S_POD_SCHEDULE_REQ, S_ADD_NODE: the only scheduler run kinds)
    } else {
        on_node(c, ep);
    }
}
K10S_HD void dispatch(Ctx& c, EvRef ep, uint32_t k) {
    if (!K10S_FULL_WAVE(XG_DISPATCH)) return;
    k = uniform_u32(k);   // wave-uniform by construction: scalar branches (see run_replica)
    if (K10S_RUNS && ((K10S_BATCH_KINDS >> k) & 1ull)) on_run_kind(c, ep, k);
    else if (k <= K10S_EV_M_GAUGE_TICK) on_metrics(c, ep);
    else if (k <= K10S_EV_AS_CREATE_GROUP_REQ) on_api_server(c, ep);
    else if (k <= K10S_EV_PS_POD_REMOVED) {
        if (k == K10S_EV_PS_CA_REQ) on_ps_ca(c, ep);
        else on_ps(c, ep);
    }
    else if (k <= K10S_EV_S_REMOVE_POD) {
        HeapEv e = *ep;
        uniform_event(e);
        on_scheduler(c, e);
    } else if (k <= K10S_EV_N_REMOVE_POD) on_node(c, ep);
    else if (k <= K10S_EV_CA_RESP) on_ca(c, ep);
    else on_hpa(c, ep);
}

// Advance the trace cursor from `cur` past the workload events that are not in this replica's
// trace (file position >= trace_prefix: k10s_replica_params.workload_prefix) and cache the head
// (time, id) in the working header.  The stream is in (time, id) order, which for workload events
// is id order, so the replica's id of a kept workload event is its scenario id minus the workload
// events skipped before it (the reference numbers only the events of the replica's own trace,
// simulator.rs:234-253); cluster events precede every workload id and keep theirs.  Returns the
// cursor; n_trace when the replica's trace is exhausted.
K10S_HD uint32_t trace_head_load(Ctx& c, uint32_t cur) {
    RepHdr& H = c.H();
    const uint32_t n = c.S().n_trace, pre = H.trace_prefix;
    uint32_t skip = H.tr_skip;
    uint32_t wp = cur < n ? c.S().trace[cur].wpos : 0u;
    while (cur < n && wp != K10S_TRACE_CLUSTER && wp >= pre) {
        skip++;
        cur++;
        wp = cur < n ? c.S().trace[cur].wpos : 0u;
    }
    if (cur < n) {
        H.tr_time = c.S().trace[cur].time;
        H.tr_seq = c.S().trace[cur].seq - (wp == K10S_TRACE_CLUSTER ? 0u : skip);
    }
    H.tr_skip = skip;
    H.trace_cursor = cur;
    return cur;
}

// ---- initialize (simulator.rs:68-275 minus the trace emission, which is the shared stream) -----
K10S_HD void perturb_pod(const Params& pr, uint32_t key, uint32_t& cpu, uint64_t& ram, double& dur) {
    uint64_t u = splitmix64(pr.seed ^ (0xD1B54A32D192ED03ull * ((uint64_t)key + 1)));
    uint32_t kd = 8 + (uint32_t)(u % 17ull);              // duration x 0.5 .. 1.5
    uint32_t kc = 12 + (uint32_t)((u >> 20) % 9ull);      // cpu x 0.75 .. 1.25
    uint32_t kr = 12 + (uint32_t)((u >> 40) % 9ull);      // ram x 0.75 .. 1.25
    dur = (dur * (double)kd) * 0.0625;
    cpu = (uint32_t)(((uint64_t)cpu * kc) >> 4);
    ram = (ram >> 4) * kr;
}

K10S_HD void init_replica(Ctx& c) {
    const Scenario* sc = &c.S();
    const Params* pr = &c.P();
    const Layout* L = &c.Ly();
    Rep v = c.V();
    const int lane = lane_id();
    const uint32_t N = sc->n_nodes, P = sc->n_pods, S = sc->n_slots, G = sc->n_groups;
    NodeState ns;
    memset(&ns, 0, sizeof ns);
    ns.as_slot = -1;
    ns.pend_def = -1;
    const NcEnt zero = {0u, 0ull};
    for (uint32_t i = lane; i < N; i += K10S_LANES) {
        nc_put(c, i, zero);
        v.node(i) = ns;
    }
    for (uint32_t i = lane; i < L->words_nodes; i += K10S_LANES) v.s_present()[i] = 0;
    if (L->front) {   // empty fronts: every node is absent, (0, 0)
        const uint32_t nbf = (N + 63u) / 64u;
        for (uint32_t i = lane; i < 8u * nbf; i += K10S_LANES) v.fr_val()[i] = 0;
        for (uint32_t i = lane; i < 8u * nbf; i += K10S_LANES) v.fr_idx()[i] = 0;
    }
    for (uint32_t i = lane; i < L->words_uids; i += K10S_LANES) v.pend_rm()[i] = 0;
    const bool perturb = pr->perturb != 0;
    k10s_pod_record* prec = v.prec();
    for (uint32_t p = lane; p < P; p += K10S_LANES) {
        uint32_t cpu = sc->pod_cpu[p];
        uint64_t ram = sc->pod_ram[p];
        double dur = sc->pod_dur[p];
        if (perturb && (sc->pod_flags[p] & POD_PERTURB)) perturb_pod(*pr, sc->pod_key[p], cpu, ram, dur);
        PodState ps;
        memset(&ps, 0, sizeof ps);
        ps.req_cpu = cpu;
        ps.req_ram = ram;
        ps.dur = dur;
        ps.s_assigned = -1;
        ps.ps_assigned = -1;
        ps.run_slot = -1;
        ps.cancel_slot = -1;
        v.pod(p) = ps;
        if (prec) {
            prec[p].t_running = __builtin_nan("");
            prec[p].t_finished = __builtin_nan("");
            prec[p].t_removed = __builtin_nan("");
            prec[p].state = 0;
            prec[p].pad = 0;
        }
    }
    SlotState ss;
    memset(&ss, 0, sizeof ss);
    ss.node = -1;
    for (uint32_t s = lane; s < S; s += K10S_LANES) {
        v.slot((int32_t)s) = ss;
        v.pool_ring()[s] = s;  // pool contexts first (FIFO), default-node components after
    }
    for (uint32_t g = lane; g < G; g += K10S_LANES) {
        GroupState gs;
        memset(&gs, 0, sizeof gs);
        v.grp()[g] = gs;
    }
    for (uint32_t i = lane; i < G * L->words_group; i += K10S_LANES) v.grp_bits()[i] = 0;
    for (uint32_t i = lane; i < 2 * sc->n_ca_groups; i += K10S_LANES) v.cag()[i] = 0;
    if (sc->ca_enabled) {
        for (uint32_t i = lane; i < L->words_pods; i += K10S_LANES) v.ca_ubits()[i] = 0;
        for (uint32_t i = lane; i < L->words_nodes; i += K10S_LANES) v.ca_live()[i] = 0;
        for (uint32_t i = lane; i < N; i += K10S_LANES) v.ps_head()[i] = -1;
    }
    wave_sync();

    // serial part (wave-uniform) on the working header
    RepHdr* h = &c.H();
    RepHdr z;
    memset(&z, 0, sizeof z);
    *h = z;
    for (int i = 0; i < 3; i++) est_reset(h->est[i]);
    // the replica's workload trace: its first workload_prefix events (0 = all)
    const uint32_t pre = pr->workload_prefix && pr->workload_prefix < sc->n_workload_trace ? pr->workload_prefix
                                                                                         : sc->n_workload_trace;
    const uint32_t first_dyn = 2 + sc->n_cluster_trace + pre;
    h->trace_prefix = pre;
    h->tr_skip = 0;
    h->counters[K10S_C_TOTAL_PODS_IN_TRACE] = sc->wl_pods_upto[pre];
    h->pods_left = (int64_t)sc->wl_pods_upto[pre];
    h->counters[K10S_C_TOTAL_NODES_IN_TRACE] = sc->total_nodes_in_trace;
    h->pool_head = 0;
    h->pool_count = sc->n_pool;
    // initialize_default_cluster (simulator.rs:303-344): present in PS, AS (own component) and S
    for (uint32_t j = 0; j < sc->n_default; j++) {
        uint32_t def = sc->default_defs[j];
        uint32_t n = sc->def_node[def];
        uint32_t slot = sc->n_pool + j;
        NodeState& nd = v.node(n);
        nd.flags |= NF_PS_PRESENT;
        if (sc->ca_enabled && sc->def_ca_origin[def]) {
            nd.flags |= NF_CA_ORIGIN;
            bit_set(v.ca_live(), n);
        }
        nd.ps_def = def;
        nd.ps_cpu = sc->def_cpu[def];
        nd.ps_ram = sc->def_ram[def];
        nd.ps_epoch = 1;
        nd.as_slot = (int32_t)slot;
        v.slot((int32_t)slot).node = (int32_t)n;
        v.slot((int32_t)slot).def = def;
        if (L->cap_gauge) {
            v.g_cpu()[slot] = sc->def_cpu[def];
            v.g_ram()[slot] = sc->def_ram[def];
        }
        const NcEnt cap = {sc->def_cpu[def], sc->def_ram[def]};
        nc_put(c, n, cap);
        fr_mark(c, n);
        if (!nc_packed(c)) {   // capacities (MostAllocated): wide layout only
            v.s_ccpu()[n] = cap.cpu;
            v.s_cram()[n] = cap.ram;
        }
        bit_set(v.s_present(), n);
    }
    h->s_node_count = sc->n_default;
    wave_sync();
    if (!nc_packed(c))   // block bounds (pruned scan): wide layout only; zero for absent nodes
        for (uint32_t b = 0; b < L->nblocks; b++) block_recompute(c, b);
    h->counters[K10S_C_NODES_READ] = 0;
    h->ps_node_count = sc->n_default;
    h->as_node_count = sc->n_default;
    h->g_cur_nodes = sc->n_default;  // simulator.rs:339-342
    h->cur_kind = 0xFFFF;
    emit0(c, K10S_EV_M_POD_METRICS_TICK, 0.0);  // id 0 (simulator.rs:156-158)
    emit0(c, K10S_EV_M_GAUGE_TICK, 0.0);        // id 1 (simulator.rs:159-161)
    h->next_seq = first_dyn;                     // trace events hold ids 2 .. first_dyn - 1
    emit0(c, K10S_EV_S_RUN_CYCLE, 0.0);          // Scheduler::start (scheduler.rs:78-81)
    emit0(c, K10S_EV_S_FLUSH, 0.0);
    if (sc->ca_enabled) emit0(c, K10S_EV_CA_TICK, 0.0);
    if (sc->hpa_enabled) emit0(c, K10S_EV_HPA_TICK, 0.0);
    trace_head_load(c, 0);
    h->status = K10S_REPLICA_RUNNING;
}

// ---- event-queue merge -------------------------------------------------------------------------

// The sorted source list.  Every event source keeps its own events in (time, id) order — a
// delay-class FIFO ring is a sorted run, the heap has its root, the trace stream its cursor — so the
// next event is the smallest of at most K10S_NSRC source heads.  The header keeps those heads sorted
// (sl[0, sl_n), non-empty sources only) and updates the list exactly where a head changes: after
// the consumed source advances, and after an emission into an empty ring or to a new heap root
// (emit marks those in sl_dirty).  The next event is then simply sl[0] — no selection over the
// sources per event (round 2 ran a 16-lane DPP minimum over all heads whenever the previous
// source's next head did not precede the runner-up: 53 % of the events at C3, measured by a shadow
// of this list on the host build, profiles/r03_selection_policy_sim.json).
K10S_HD bool sl_less(int64_t ka, uint32_t sa, int64_t kb, uint32_t sb) { return ka < kb || (ka == kb && sa < sb); }

// Current head (time key, id) of source q; false if q is empty.
K10S_HD bool src_head(Ctx& c, uint32_t q, uint32_t ntr, int64_t& k, uint32_t& s) {
    const RepHdr& H = c.H();
    if (q < (uint32_t)K10S_NFQ) {
        const uint32_t hd = H.fq[q].head, tl = H.fq[q].tail;
        const HeapEv& t = H.fq_win[q * K10S_FQW + (hd & (K10S_FQW - 1))];
        k = total_key(t.time);
        s = t.seq;
        return hd != tl;
    }
    if (q == (uint32_t)SRC_TRACE) {
        k = total_key(H.tr_time);
        s = H.tr_seq;
        return H.trace_cursor < ntr;
    }
    k = total_key(H.heap_top.time);
    s = H.heap_top.seq;
    return H.heap_size > 0;
}

// Replace source q's entry by its new head (key, seq), or drop it (has == false).  Device: one
// 16-B LDS read per lane (lane i = entry i), the new positions from two ballots, one scattered
// 16-B write per kept entry and one for the new entry: no serial walk.
K10S_HD void sl_update(Ctx& c, uint32_t q, bool has, int64_t key, uint32_t seq) {
    RepHdr& H = c.H();
#if K10S_DEVICE
    if (!K10S_FULL_WAVE(XG_SL_UPDATE)) return;
    const uint32_t n = uniform_u32(H.sl_n);
    const uint32_t lane = (uint32_t)lane_id();
    SrcEnt E;
    E.key = 0x7FFFFFFFFFFFFFFFll;
    E.seq = 0xFFFFFFFFu;
    E.src = 0xFFFFFFFFu;
    if (lane < n) E = H.sl[lane];
    const bool keep = lane < n && E.src != q;
    const bool less = keep && sl_less(E.key, E.seq, key, seq);
    const uint64_t mk = __ballot(keep);
    const uint32_t p = (uint32_t)__popcll(__ballot(less));   // the new entry's index
    const uint32_t before = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
    const uint32_t idx = before + ((has && !less) ? 1u : 0u);
    if (keep) H.sl[idx] = E;
    if (has && lane == 0) {
        SrcEnt N;
        N.key = key;
        N.seq = seq;
        N.src = q;
        H.sl[p] = N;
    }
    H.sl_n = (uint32_t)__popcll(mk) + (has ? 1u : 0u);
#else
    uint32_t n = H.sl_n, w = 0;
    for (uint32_t i = 0; i < n; i++)
        if (H.sl[i].src != q) H.sl[w++] = H.sl[i];
    n = w;
    if (has) {
        uint32_t i = n;
        while (i > 0 && sl_less(key, seq, H.sl[i - 1].key, H.sl[i - 1].seq)) {
            H.sl[i] = H.sl[i - 1];
            i--;
        }
        K10S_HSTAT(HS_SLPOS0 + (i < 3 ? i : 3));
        H.sl[i].key = key;
        H.sl[i].seq = seq;
        H.sl[i].src = q;
        n++;
    }
    H.sl_n = n;
#endif
}
K10S_HD void sl_refresh(Ctx& c, uint32_t q, uint32_t ntr) {
    int64_t k;
    uint32_t s;
    const bool has = src_head(c, q, ntr, k, s);
    sl_update(c, q, has, uniform_u64((uint64_t)k), uniform_u32(s));
}
// Apply the head changes emissions made since the last update.
K10S_HD void sl_apply_dirty(Ctx& c, uint32_t ntr) {
    uint32_t d = uniform_u32(c.H().sl_dirty);
    if (!d) return;
    c.H().sl_dirty = 0;
    do {
        const uint32_t q = (uint32_t)__builtin_ctz(d);
        d &= d - 1;
        K10S_HSTAT(HS_SL_DIRTY);
        sl_refresh(c, q, ntr);
    } while (d);
}
// Build the list from scratch (start of a launch: the header may come from anywhere).
K10S_HD void sl_rebuild(Ctx& c, uint32_t ntr) {
    c.H().sl_n = 0;
    c.H().sl_dirty = 0;
    for (uint32_t q = 0; q < (uint32_t)K10S_NSRC; q++) sl_refresh(c, q, ntr);
}

// Refill a drained delay-class window from the HBM ring: positions [hd, hd + min(W, tail - hd)),
// one 32-B entry per lane, so a burst of FIFO events costs one memory round trip per K10S_FQW pops.
K10S_HD void fq_refill(Ctx& c, int cls, uint32_t hd) {
    if (!K10S_FULL_WAVE(XG_FQ_REFILL)) return;
    RepHdr& H = c.H();
    const uint32_t cap = c.Ly().cap_fq;
    const uint32_t avail = H.fq[cls].tail - hd;
    const uint32_t n = avail < K10S_FQW ? avail : K10S_FQW;
    const HeapEv* ring = c.V().fq() + (uint32_t)cls * cap;
    for (uint32_t i = (uint32_t)lane_id(); i < n; i += K10S_LANES)
        H.fq_win[(uint32_t)cls * K10S_FQW + ((hd + i) & (K10S_FQW - 1))] = ring[(hd + i) & (cap - 1)];
    H.fq[cls].wend = hd + n;
}

// (Round 3 measured an asynchronous window refill — an LDS-DMA copy of the next ring entries into
// freed window slots, waited for when the head reaches them — and did not keep it: C3 1,242 ->
// 1,272 ms, the vmcnt(0) wait at the first copied entry also waits for the previous handler's
// stores; profiles/r03_k5_fq_prefetch_ab.json.)
// Remove the head event of source src (sl[0]) and move the source's entry in the source list to
// its new head; a FIFO takes its next head from its window.  When the new
// head still precedes sl[1], only sl[0]'s key is rewritten (tuning knob, semantics-neutral).
K10S_HD void sl_after_consume(Ctx& c, int src, bool has, int64_t key, uint32_t seq);
K10S_HD void consume_source(Ctx& c, int src, uint32_t ntr) {
    src = (int)uniform_u32((uint32_t)src);   // wave-uniform by construction: scalar branches (see run_replica)
    RepHdr& H = c.H();
    bool has;
    int64_t key = 0;
    uint32_t seq = 0;
    K10S_HSTAT(HS_EVENTS);
    if (src == SRC_TRACE) {
        K10S_HSTAT(HS_TRACE_POP);
        const uint32_t cur = trace_head_load(c, H.trace_cursor + 1);
        has = cur < ntr;
        if (has) {
            key = total_key(H.tr_time);
            seq = H.tr_seq;
        }
    } else if (src == SRC_HEAP) {
        const uint64_t t_hp = prof_now();
        heap_pop(c);
        K10S_HSTAT(HS_HEAP_POP);
        K10S_PROF_ADD(c, PROF_HEAPPOP, t_hp);
        K10S_PROF_COUNT(c, PROF_NHEAPPOP);
        has = src_head(c, SRC_HEAP, ntr, key, seq);
    } else {
        const uint32_t hd = H.fq[src].head + 1, tl = H.fq[src].tail, we = H.fq[src].wend;
        K10S_HSTAT(HS_POP_CLS0 + src);
        H.fq[src].head = hd;
        has = hd != tl;
        K10S_HSTAT(HS_FIFO_POP);
        if (has) {
            if (hd == we) {
                fq_refill(c, src, hd);
                K10S_HSTAT(HS_REFILL);
                K10S_HSTAT(HS_REFILL_CLS0 + src);
            }
            const HeapEv& t = H.fq_win[(uint32_t)src * K10S_FQW + (hd & (K10S_FQW - 1))];
            key = total_key(t.time);
            seq = t.seq;
        }
    }
    sl_after_consume(c, src, has, key, seq);
}

// The consumed source src (sl[0]) has its new head (key, seq), or is empty (!has): reposition it.
K10S_HD void sl_after_consume(Ctx& c, int src, bool has, int64_t key, uint32_t seq) {
    RepHdr& H = c.H();
    key = (int64_t)uniform_u64((uint64_t)key);
    seq = uniform_u32(seq);
    // src is sl[0]: while its new head still precedes the second source (47 % of the events at C3,
    // profiles/r03_selection_policy_sim.json) only sl[0]'s key changes — no lane-parallel update
    if (has) {
        // sl[1] is read whether or not it is live (LDS; ignored when n <= 1), so the three reads
        // issue together
        const int64_t k1 = (int64_t)uniform_u64((uint64_t)H.sl[1].key);
        const uint32_t s1 = uniform_u32(H.sl[1].seq);
        const uint32_t n = uniform_u32(H.sl_n);
        const bool stays = n <= 1 || sl_less(key, seq, k1, s1);
        if (stays) {
            H.sl[0].key = key;
            H.sl[0].seq = seq;
            K10S_HSTAT(HS_SL_FAST);
            return;
        }
    }
    K10S_HSTAT(HS_SL_UPDATE);
    sl_update(c, (uint32_t)src, has, key, seq);
}

// Does some node of the scheduler cache fit a (cpu, ram) request (Fit::filter, plugin.rs:34-45)?
// Lane-parallel over node indices with an early exit; a zero request never schedules
// (RequestedResourcesAreZeros, kube_scheduler.rs:74-76).
K10S_HD bool cache_fits(Ctx& c, uint32_t rc, uint64_t rr) {
    if (!K10S_FULL_WAVE(XG_CACHE_FITS)) return true;
    if (rc == 0 && rr == 0) return false;
    const uint32_t N = c.S().n_nodes;
    const uint64_t* pres = c.V().s_present();
    for (uint32_t base = 0; base < N; base += K10S_LANES) {
        const uint32_t n = base + (uint32_t)lane_id();
        bool f = false;
        if (n < N && bit_test(pres, n)) {
            const NcEnt v = nc_get(c, n);
            f = rc <= v.cpu && rr <= v.ram;
        }
        if (wave_any(f)) return true;
    }
    return false;
}

// Stall guard (opt-in, k10s_capacities.stall_guard), evaluated after a gauge tick: the trace is
// exhausted, the heap holds only the four periodic ticks (pod metrics, gauge, scheduling cycle,
// flush; a pending pod finish, even a lazily canceled one, counts as progress), every delay-class
// ring is empty, the action queue is empty and neither autoscaler runs.  Then no node's
// allocatable can change again.  The replica is stalled only if, in addition, no live entry of the
// unschedulable map fits any node of that frozen cache: then every retry fails as before and the
// replica would cycle until max_time (TIME_LIMIT) without terminating another pod.  (With the
// conditional move, scheduler.rs:210-233, a pod that fits only the resources freed by several
// finishes together is not moved by any of them and waits for the 300-s flush, 188-203: such an
// entry fits the cache now and keeps the replica running.)
K10S_HD bool replica_stalled(Ctx& c) {
    const RepHdr& H = c.H();
    if (H.pods_left <= 0) return false;
    if (H.trace_cursor < c.S().n_trace || H.heap_size != 4 || H.aq_size != 0) return false;
    if (c.S().ca_enabled || c.S().hpa_enabled) return false;
    for (int q = 0; q < K10S_NFQ; q++)
        if (H.fq[q].head != H.fq[q].tail) return false;
    const QInfo* d = c.V().uq();
    const uint32_t n = uniform_u32(H.uq_size);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t p = uniform_u32(d[i].pod);
        if (!pod_in_s(c, p)) continue;  // stale entry of a deleted pod: never moved again
        if (cache_fits(c, uniform_u32(c.V().pod(p).req_cpu), uniform_u64(c.V().pod(p).req_ram))) return false;
    }
    return true;
}

// ---- the event loop -----------------------------------------------------------------------------
// Wave priorities (s_setprio) so that the replicas of one SIMD drain together.  The instruction
// arbiter prefers the oldest wave among equal priorities, so with 8 identical replicas per SIMD the
// oldest finished at 63 % of the launch and the youngest at 100 % (tools/wall_spread.py,
// profiles/r02_v7_wall_spread_*.json): the SIMD ran the last third with fewer and fewer waves.
// Every 2^K10S_FAIR_SHIFT events a wave adds its progress to a per-SIMD board and picks a priority:
// random 1..2 while within K10S_FAIR_BAND events of its SIMD's mean, 3 when behind by more, 0 when
// ahead by more.  Measured against the alternatives (profiles/r02_v7_fair_ab.json, C3 ms): none
// 2,089; random 0..3 1,836; rotation by SIMD slot 1,871-1,913; strict least-progress-first 1,873
// (every replica ends together but the SIMD issues less while 8 waves compete evenly); this banded
// hybrid 1,734.  Scheduling hints only: no effect on any result.
#ifndef K10S_FAIR_SHIFT
#define K10S_FAIR_SHIFT 6
#endif
#ifndef K10S_FAIR_BAND
#define K10S_FAIR_BAND 512
#endif
#define K10S_FAIR_KEYS 4096   // XCC x SE x SH x CU x SIMD
#if defined(__HIP__)
__device__ uint32_t k10s_fair_board[2 * K10S_FAIR_KEYS];   // zeroed before every run launch
#endif
K10S_HD void fair_priority(uint64_t done) {
#if K10S_DEVICE
    if ((done & ((1ull << K10S_FAIR_SHIFT) - 1)) != 0) return;
    if (!K10S_FULL_WAVE(XG_FAIR)) return;
    // the waves of one SIMD (HW_ID + XCC_ID key) add their event counts to a per-SIMD board (vector
    // atomics by lanes 0/1 on distinct words)
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) & 7u;
    const uint32_t key = (((xcc * 4u + ((hw >> 13) & 3u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) * 4u +
                         ((hw >> 4) & 3u);
    const int lane = lane_id();
    const uint32_t inc = 1u << K10S_FAIR_SHIFT;
    uint32_t got = 0;
    if (lane < 2) {
        uint32_t* w = lane == 0 ? &k10s_fair_board[key] : &k10s_fair_board[K10S_FAIR_KEYS + key];
        got = atomicAdd(w, lane == 0 ? inc : (done == 0 ? 1u : 0u));
    }
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)got, 0) + inc;
    uint32_t nw = (uint32_t)__builtin_amdgcn_readlane((int)got, 1) + (done == 0 ? 1u : 0u);
    nw = nw ? nw : 1u;
    const int64_t lag = (int64_t)(tot / nw) - (int64_t)(done + inc);
    const uint32_t rnd = 1u + (uint32_t)(splitmix64(((uint64_t)blockIdx.x << 32) ^ (done >> K10S_FAIR_SHIFT)) >> 63);
    const uint32_t pr = lag > (int64_t)K10S_FAIR_BAND ? 3u : lag < -(int64_t)K10S_FAIR_BAND ? 0u : rnd;
    switch (pr) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
#else
    (void)done;
#endif
}
// Drop the heap's head, a lazily canceled pod finish, and move the heap's source-list entry to its
// new head.  Out of line on purpose: inlined into the selection loop below, sl_update's lane-0
// store (`has && lane == 0`) was threaded into the loop's back edge in the K10S_PROF build, which
// the structurizer then compiled as a divergent loop (exec-masked flow blocks around heap_pop); the
// first stale skip of c5_autoscaled replica 53 never left it.  A
// call keeps every lane-divergent branch of the skip inside the callee, so the selection loop has
// only uniform (scalar) branches in every build.
K10S_HD_NOINL void drop_stale_head(Ctx& c, uint32_t ntr) {
    c.H().stale_fin -= 1;
    heap_pop(c);
    sl_refresh(c, SRC_HEAP, ntr);
}
// ---- runs of one event kind, handled together (round 5) -------------------------------------------
// The C3 workload delivers many events in runs: the 13-14 pods of an integer-second arrival burst
// pass the api server, storage and the scheduler's queue as three runs of 13-14 consecutive events of
// one kind, from one source, at one time (AS_CREATE_POD_REQ from the trace, PS_CREATE_POD_REQ from the
// as-to-ps ring, S_POD_SCHEDULE_REQ from the ps-to-sched ring: mean run 13.65), and the 4,096 nodes of
// the trace are created at t = 0 as five runs of 4,096 (AS_CREATE_NODE_REQ, PS_CREATE_NODE_REQ,
// AS_CREATE_NODE_RESP, PS_NODE_ADDED, S_ADD_NODE).  Handling a run event by event pays the
// selection, the dispatch and the consume once per event; here they are paid once per run (of up to
// 64 events) and the K handlers run as K lanes.
//
// Why it is exact.  The run is the next K events in dslab (time, id) order: consecutive heads of source
// src, all of kind k and time t, all before the head of the second source in the source list (sl[1]),
// so no other source delivers in between.  Every event a handler of the run emits has time t + d >= t
// and an id larger than every pending id (ids are handed out in emission order), so it is ordered after
// the whole run and cannot interleave with it.  The handlers of these kinds touch their own pod's or
// node's line, header counters that commute, slots taken from the pool ring in event order, presence
// bits set with atomics, and the emission sequence; the batch hands out ids next_seq + i in event order
// (one emission per event, as the serial handlers do) and appends to the target ring in that order.
// What the serial path would do differently is excluded before anything is written — a reference panic
// (a pod already in storage, a node already present / not pending / missing, an empty node pool, or
// one pod or node twice in the run), a full ring or a run that would break its ring's time order
// (those emissions go to the heap), an id overflow, a full action queue, a cluster autoscaler or the
// pruned scan's block bounds (their per-node upkeep), a non-empty unschedulable map (a node added with
// pods waiting moves them) — and then the run is not batched: the loop takes its events one by one.
// The termination rule cannot fire inside a run (none of these kinds terminates a pod), and the time
// limit and event budget are checked for the run's time and length by the caller.
#define K10S_RUN_MAX 64
// i = the run event this lane handles: one pass of the lanes below K on the device, a loop on the host
#if K10S_DEVICE
#define K10S_FOR_RUN(i, K) for (uint32_t i = (uint32_t)lane_id(), i##_1 = 0; i##_1 == 0 && i < (K); i##_1 = 1)
#else
#define K10S_FOR_RUN(i, K) for (uint32_t i = 0; i < (K); i++)
#endif
K10S_HD bool run_kind(uint32_t k) {
    return k == K10S_EV_AS_CREATE_POD_REQ || k == K10S_EV_PS_CREATE_POD_REQ || k == K10S_EV_S_POD_SCHEDULE_REQ ||
           k == K10S_EV_AS_CREATE_NODE_REQ || k == K10S_EV_PS_CREATE_NODE_REQ || k == K10S_EV_AS_CREATE_NODE_RESP ||
           k == K10S_EV_PS_NODE_ADDED || k == K10S_EV_S_ADD_NODE;
}
// Event i of a run at source src: FIFO position head + i (its LDS window below wend, the HBM ring
// above), or trace position trace_cursor + i (a and b as the loop materializes a trace event).  ok =
// false when it does not exist or is a workload event outside this replica's trace (its id would shift).
struct RunEv {
    double time, x;
    uint32_t seq, kind, a, b;
    bool ok;
};
K10S_HD RunEv run_ev(Ctx& c, int src, uint32_t i) {
    const RepHdr& H = c.H();
    RunEv r;
    r.time = 0.0;
    r.x = 0.0;
    r.seq = 0;
    r.kind = 0xFFFFu;
    r.a = 0;
    r.b = 0;
    r.ok = false;
    if (src == SRC_TRACE) {
        const uint32_t cur = H.trace_cursor + i;
        if (cur < c.S().n_trace) {
            const TraceEv t = c.S().trace[cur];
            const bool wl = t.wpos != K10S_TRACE_CLUSTER;
            r.ok = !wl || t.wpos < H.trace_prefix;
            r.time = t.time;
            r.seq = t.seq - (wl ? H.tr_skip : 0u);
            r.kind = t.kind;
            r.a = t.arg;
            if (t.kind == K10S_EV_AS_CREATE_NODE_REQ) {   // as run_replica materializes it
                r.a = c.S().def_node[t.arg];
                r.b = t.arg;
            }
        }
    } else {
        const uint32_t hd = H.fq[src].head, tl = H.fq[src].tail, we = H.fq[src].wend;
        if (i < tl - hd) {
            const uint32_t pos = hd + i;
            HeapEv e;
            if (pos - hd < we - hd) e = H.fq_win[(uint32_t)src * K10S_FQW + (pos & (K10S_FQW - 1))];
            else e = c.V().fq()[(uint32_t)src * c.Ly().cap_fq + (pos & (c.Ly().cap_fq - 1))];
            r.ok = true;
            r.time = e.time;
            r.x = e.x;
            r.seq = e.seq;
            r.kind = e.kind;
            r.a = e.a;
            r.b = e.b;
        }
    }
    return r;
}

// Called by the handler of the current event (kind k, at the head of its source, which is sl[0]; the
// clock is its time): handle the run it starts, K >= 2 events, and return K, or 0 when the events must
// go one by one (nothing was written then).  On return the K handlers have run, events 1..K-1 are
// logged and counted, and the source is advanced past events 0..K-2: the event loop's own consume of
// the current event then removes the last one (the loop itself is unchanged: a call in its body would
// re-spill its live registers around every event; round 5 measured that layout at -9.6 % on C3).
K10S_HD_NOINL uint32_t run_batch(Ctx& c, uint32_t k) {
    RepHdr& H = c.H();
    k = uniform_u32(k);
    const uint32_t fl = uniform_u32(H.run_flags);
    // budgeted launches count events one by one; the termination rule is checked before every event
    // (it cannot fire inside a run while pods are left, or in until-time mode)
    if (!(fl & 1u) || (!(fl & 2u) && (int64_t)uniform_u64((uint64_t)H.pods_left) <= 0)) return 0;
    const int src = (int)uniform_u32(H.sl[0].src);
    if (src == SRC_HEAP) return 0;
    const double t = uniform_f64(H.clock);
    const uint32_t kmax = K10S_RUN_MAX;
    const int64_t kt = total_key(t);
    // the second source's head bounds the run
    const uint32_t sn = uniform_u32(H.sl_n);
    const int64_t k1 = sn >= 2 ? (int64_t)uniform_u64((uint64_t)H.sl[1].key) : 0x7FFFFFFFFFFFFFFFll;
    const uint32_t s1 = sn >= 2 ? uniform_u32(H.sl[1].seq) : 0xFFFFFFFFu;
    const uint32_t lim = kmax < K10S_RUN_MAX ? kmax : K10S_RUN_MAX;
    // ---- the run's length: the leading events that are of kind k, at time t, before sl[1]
    uint32_t K = 0;
#if K10S_DEVICE
    {
        const uint32_t lane = (uint32_t)lane_id();
        bool in = false;
        if (lane < lim) {
            const RunEv r = run_ev(c, src, lane);
            in = r.ok && r.kind == k && total_key(r.time) == kt && sl_less(kt, r.seq, k1, s1);
        }
        const uint64_t m = ~__ballot(in);
        K = m ? (uint32_t)__builtin_ctzll(m) : 64u;
    }
#else
    while (K < lim) {
        const RunEv r = run_ev(c, src, K);
        if (!(r.ok && r.kind == k && total_key(r.time) == kt && sl_less(kt, r.seq, k1, s1))) break;
        K++;
    }
#endif
    K = uniform_u32(K);
    if (K < 2) return 0;
    K10S_HSTAT(HS_RUN_REFUSED);   // (taken back below once the run is handled)
    // ---- everything the serial path would do differently: then no batch
    const uint32_t seq0 = uniform_u32(H.next_seq);
    if ((uint64_t)seq0 + K > 0xFFFFFFFFull) return 0;   // an id would reach 2^32 - 1 (K10S_ERR_SEQ_OVERFLOW)
    const Params& pr = c.P();
    const Scenario& S = c.S();
    int cls = -1;     // the emissions' delay class
    double d = 0.0;
    uint32_t ek = 0;  // and kind
    bool uniq = false;   // the run's pods / nodes must be distinct
    switch (k) {
    case K10S_EV_AS_CREATE_POD_REQ:
        cls = FQ_AS_TO_PS, d = pr.as_to_ps_network_delay, ek = K10S_EV_PS_CREATE_POD_REQ;
        break;
    case K10S_EV_PS_CREATE_POD_REQ:
        cls = FQ_PS_TO_SCHED, d = pr.ps_to_sched_network_delay, ek = K10S_EV_S_POD_SCHEDULE_REQ, uniq = true;
        break;
    case K10S_EV_S_POD_SCHEDULE_REQ:
        if (uniform_u32(H.aq_size) + K > c.Ly().cap_aq) return 0;
        break;
    case K10S_EV_AS_CREATE_NODE_REQ:
        cls = FQ_AS_TO_PS, d = pr.as_to_ps_network_delay, ek = K10S_EV_PS_CREATE_NODE_REQ, uniq = true;
        break;
    case K10S_EV_PS_CREATE_NODE_REQ:
        if (S.ca_enabled) return 0;   // CA-origin nodes: shared bitmap words, assignment lists
        cls = FQ_AS_TO_PS, d = pr.as_to_ps_network_delay, ek = K10S_EV_AS_CREATE_NODE_RESP, uniq = true;
        break;
    case K10S_EV_AS_CREATE_NODE_RESP:
        if (uniform_u32(H.pool_count) < K) return 0;   // node_component_pool.rs:56-59
        cls = FQ_AS_TO_PS, d = pr.as_to_ps_network_delay, ek = K10S_EV_PS_NODE_ADDED, uniq = true;
        break;
    case K10S_EV_PS_NODE_ADDED:
        cls = FQ_PS_TO_SCHED, d = pr.ps_to_sched_network_delay, ek = K10S_EV_S_ADD_NODE;
        break;
    default:   // K10S_EV_S_ADD_NODE
        // with pods in the unschedulable map each addition moves some (scheduler.rs:391-405); the wide
        // layout keeps capacities and (pruned scan) block bounds per node
        if (uniform_u32(H.uq_size) != 0 || !nc_packed(c) || c.Ly().pruned) return 0;
        uniq = true;
        break;
    }
    const uint32_t cap = c.Ly().cap_fq;
    const double te = t + d;
    uint32_t fhd = 0, ftl = 0, fwe = 0;
    if (cls >= 0) {
        fhd = uniform_u32(H.fq[cls].head);
        ftl = uniform_u32(H.fq[cls].tail);
        fwe = uniform_u32(H.fq[cls].wend);
        const double last = uniform_f64(H.fq[cls].last);
#if !K10S_TIME_KEY_ID
        if (!(d >= 0.0)) return 0;   // a negative delay panics in emit (signed-time kernel copy)
#endif
        // room: the run's own slots count when it is consumed from the target ring itself (storage's
        // node creation answers the api server on the ring that brought the request) — each lane reads
        // its run event before any lane writes, and emission i lands on run event i - free's slot, so
        // the overlap is safe; at t = 0 that ring holds all 4,096 node requests, which the serial path
        // answers through the heap
        const uint32_t room = cap - (ftl - fhd) + (src == cls ? K : 0u);
        if (!cap || room < K || (ftl != fhd && total_key(te) < total_key(last))) return 0;
    }
    {
        bool bad = false;
        K10S_FOR_RUN(i, K) {
            const RunEv r = run_ev(c, src, i);
            if (k == K10S_EV_PS_CREATE_POD_REQ) {
                bad |= (c.V().pod(r.a).flags & PF_IN_PS) != 0;   // persistent_storage.rs:89-94
            } else if (k == K10S_EV_PS_CREATE_NODE_REQ) {
                bad |= (c.V().node(r.a).flags & NF_PS_PRESENT) != 0;   // persistent_storage.rs:76-81
            } else if (k == K10S_EV_AS_CREATE_NODE_RESP) {
                const NodeState& N = c.V().node(r.a);   // api_server.rs:98-101, 73-78
                bad |= N.pend_def < 0 || N.as_slot >= 0;
            } else if (k == K10S_EV_PS_NODE_ADDED) {
                bad |= (c.V().node(r.a).flags & NF_PS_PRESENT) == 0;
            }
            if (uniq) {   // one pod / node twice: the serial path would see the first one's writes
#if K10S_DEVICE
                for (uint32_t j = 0; j < K; j++) bad |= j < i && (uint32_t)__builtin_amdgcn_readlane((int)r.a, (int)j) == r.a;
#else
                for (uint32_t j = 0; j < i; j++) bad |= run_ev(c, src, j).a == r.a;
#endif
            }
        }
        if (wave_any(bad)) return 0;
    }
    // ---- the K handlers, one per lane
    const uint32_t cap_log = c.Ly().cap_log;
    const uint32_t log0 = uniform_u32(H.log_n) - 1u;   // event 0 was logged by the event loop
    const uint32_t pool_head = uniform_u32(H.pool_head);
    uint32_t cnt = 0;   // per lane: PF_UNSCHED pods (PS_CREATE_POD_REQ) / newly present nodes (S_ADD_NODE)
    uint64_t fbits = 0;  // S_ADD_NODE: the blocks whose front the lane's node changes (fr_mark)
    K10S_FOR_RUN(i, K) {
        const RunEv r = run_ev(c, src, i);
        const bool node_kind = k != K10S_EV_AS_CREATE_POD_REQ && k != K10S_EV_PS_CREATE_POD_REQ &&
                               k != K10S_EV_S_POD_SCHEDULE_REQ;
        if (cap_log && i > 0 && log0 + i < cap_log) {
            k10s_log_entry le;
            le.time = r.time;
            le.seq = r.seq;
            le.kind = (uint16_t)k;
            le.slot = -1;
            le.pod = node_kind ? -1 : (int32_t)r.a;
            le.node = node_kind ? (int32_t)r.a : -1;
            c.V().log()[log0 + i] = le;
        }
        uint32_t eb = 0;   // the emission's b and x
        double ex = 0.0;
        switch (k) {
        case K10S_EV_PS_CREATE_POD_REQ: {
            PodState& P = c.V().pod(r.a);
            const uint8_t pf = P.flags;
            P.flags = (uint8_t)(pf | PF_IN_PS);
            cnt += (pf & PF_UNSCHED) ? 1u : 0u;
            P.ps_assigned = -1;
            if (c.V().prec()) c.V().prec()[r.a].state = 1;
            break;
        }
        case K10S_EV_S_POD_SCHEDULE_REQ:
            c.V().pod(r.a).sflag = PF_IN_S;
            c.V().pod(r.a).s_assigned = -1;
            break;
        case K10S_EV_AS_CREATE_NODE_REQ:   // api_server.rs:132-137
            c.V().node(r.a).pend_def = (int32_t)r.b;
            eb = r.b;
            break;
        case K10S_EV_PS_CREATE_NODE_REQ: {   // persistent_storage.rs:188-195 (no CA)
            NodeState& N = c.V().node(r.a);
            N.flags = (uint8_t)((N.flags & ~NF_CA_ORIGIN) | NF_PS_PRESENT);
            N.ps_def = r.b;
            N.ps_cpu = S.def_cpu[r.b];
            N.ps_ram = S.def_ram[r.b];
            N.ps_epoch += 1;
            break;
        }
        case K10S_EV_AS_CREATE_NODE_RESP: {   // handle_create_node (api_server.rs:96-115): slots in event order
            NodeState& N = c.V().node(r.a);
            const uint32_t def = (uint32_t)N.pend_def;
            N.pend_def = -1;
            const uint32_t slot = c.V().pool_ring()[(pool_head + i) % S.n_slots];
            c.V().slot((int32_t)slot).node = (int32_t)r.a;
            c.V().slot((int32_t)slot).def = def;
            N.as_slot = (int32_t)slot;
            if (c.Ly().cap_gauge) {
                c.V().g_cpu()[slot] = S.def_cpu[def];
                c.V().g_ram()[slot] = S.def_ram[def];
            }
            ex = r.time;
            break;
        }
        case K10S_EV_PS_NODE_ADDED:   // persistent_storage.rs:197-210
            eb = c.V().node(r.a).ps_cpu;
            ex = u2f(c.V().node(r.a).ps_ram);
            break;
        case K10S_EV_S_ADD_NODE: {   // scheduler.rs:391-405 (packed cache, empty unschedulable map)
            const NcEnt ent = {r.b, f2u(r.x)};
            nc_put(c, r.a, ent);
            fbits |= 1ull << (r.a >> 6);
            const uint64_t bit = 1ull << (r.a & 63u);
#if K10S_DEVICE
            const uint64_t old = atomicOr((unsigned long long*)&c.V().s_present()[r.a >> 6], (unsigned long long)bit);
#else
            const uint64_t old = c.V().s_present()[r.a >> 6];
            c.V().s_present()[r.a >> 6] = old | bit;
#endif
            cnt += (old & bit) ? 0u : 1u;
            break;
        }
        default:
            break;
        }
        if (cls >= 0) {   // its one emission: id seq0 + i, ring position ftl + i
            HeapEv e;
            e.time = te;
            e.seq = seq0 + i;
            e.kind = (uint16_t)ek;
            e.slot = -1;
            e.a = r.a;
            e.b = eb;
            e.x = ex;
            c.V().fq()[(uint32_t)cls * cap + ((ftl + i) & (cap - 1))] = e;
            // the window holds the whole ring and has room: the first entries go there as well
            if (fwe == ftl && (ftl - fhd) + i < K10S_FQW) H.fq_win[(uint32_t)cls * K10S_FQW + ((ftl + i) & (K10S_FQW - 1))] = e;
        }
    }
    wave_sync();
    if (cap_log) {   // (the loop logged event 0 at log0, or flagged the overflow)
        if (log0 + K <= cap_log) H.log_n = log0 + K;
        else {
            H.log_n = log0 + 1u < cap_log ? cap_log : log0 + 1u;
            H.flags |= 1u;
        }
    }
    switch (k) {
    case K10S_EV_AS_CREATE_POD_REQ: H.g_cur_pods += K; break;   // api_server.rs:151-155
    case K10S_EV_PS_CREATE_POD_REQ: H.unsched_missing -= wave_sum_u32(cnt); break;
    case K10S_EV_AS_CREATE_NODE_REQ: H.g_cur_nodes += K; break;
    case K10S_EV_PS_CREATE_NODE_REQ: H.ps_node_count += K; break;
    case K10S_EV_AS_CREATE_NODE_RESP:
        H.pool_head = (pool_head + K) % S.n_slots;
        H.pool_count -= K;
        H.as_node_count += K;
        break;
    case K10S_EV_PS_NODE_ADDED: H.counters[K10S_C_PROCESSED_NODES] += K; break;
    case K10S_EV_S_ADD_NODE:
        H.s_node_count += wave_sum_u32(cnt);
        if (K10S_FRONT && c.Ly().front) H.fr_dirty |= wave_or_u64(fbits);
        break;
    default: break;
    }
    if (cls >= 0) {
        if (fwe == ftl && ftl - fhd < K10S_FQW) {
            const uint32_t room = K10S_FQW - (ftl - fhd);
            H.fq[cls].wend = ftl + (K < room ? K : room);
        }
        if (ftl == fhd) sl_mark(H, (uint32_t)cls);   // the ring was empty: a new head (source list)
        H.fq[cls].tail = ftl + K;
        H.fq[cls].last = te;
        H.next_seq = seq0 + K;
    }
    if (k == K10S_EV_S_POD_SCHEDULE_REQ) {
        // The K pushes in event order (the Rust BinaryHeap's sifts depend on the order).  Push i puts its
        // entry (key t) at position n + i and sift_up stops at once when its parent's timestamp is <= t
        // (queue.rs:29-33: `elem <= parent`); a parent inside the run has key t itself.  When that holds
        // for every push whose parent is an older entry, the K pushes are K appends: one lane each, the
        // parents read in one round trip instead of one dependent round trip per push.
        const uint32_t n0 = uniform_u32(H.aq_size);
        bool moves = false;
        K10S_FOR_RUN(i, K) {
            const uint32_t pos = n0 + i;
            if (pos > 0 && (pos - 1u) / 2u < n0) moves |= total_key(aq_raw(c, (pos - 1u) / 2u).timestamp) > kt;
        }
        if (!wave_any(moves)) {
            K10S_FOR_RUN(i, K) {
                QInfo q;
                q.timestamp = t;
                q.initial = t;
                q.attempts = 1;
                q.pod = run_ev(c, src, i).a;
                aq_put(c, n0 + i, q);
            }
            // sorted mode (aq_push) survives one push strictly above the newest; K equal keys leave it
            const bool srt = K10S_AQ_SORTED && K == 1u &&
                             (n0 == 0u || (uniform_u32(H.aq_sorted) != 0u && kt > (int64_t)uniform_u64((uint64_t)H.aq_last)));
            H.aq_sorted = srt ? 1u : 0u;
            H.aq_last = kt;
            H.aq_size = n0 + K;
            K = uniform_u32(K);
            goto pushed;
        }
    }
    if (k == K10S_EV_S_POD_SCHEDULE_REQ) {
#if K10S_DEVICE
        const uint32_t lane_a = (uint32_t)lane_id() < K ? run_ev(c, src, (uint32_t)lane_id()).a : 0u;
#endif
        for (uint32_t i = 0; i < K; i++) {
#if K10S_DEVICE
            const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)lane_a, (int)i);
#else
            const uint32_t p = run_ev(c, src, i).a;
#endif
            QInfo q;
            q.timestamp = t;
            q.initial = t;
            q.attempts = 1;
            q.pod = p;
            aq_push(c, q);
        }
    }
pushed:
    // ---- advance the source past events 0..K-2 (the loop's consume removes event K-1)
    if (src == SRC_TRACE) {
        H.trace_cursor = uniform_u32(H.trace_cursor) + (K - 1u);   // no skipped entry inside a run
    } else {
        const uint32_t hd = uniform_u32(H.fq[src].head) + (K - 1u);
        const uint32_t we = uniform_u32(H.fq[src].wend);
        H.fq[src].head = hd;
        // the loop's consume refills the window when the head reaches its end: keep the head inside it
        if ((int32_t)(hd - we) >= 0) fq_refill(c, src, hd);
    }
    H.counters[K10S_C_EVENTS] += K - 1u;
#if K10S_PROF
    H.prof[K10S_PROF_KIND0 + K10S_EV_NUM_KINDS + k] += K - 1u;
#endif
#if !K10S_DEVICE && defined(K10S_HOST_STATS)
    k10s_host_stats[HS_RUN_REFUSED] -= 1;
    k10s_host_stats[HS_RUNS] += 1;
    k10s_host_stats[HS_RUN_EVENTS] += K;
    k10s_host_stats[HS_EVENTS] += K - 1;
#endif
    return K;
}

// ---- windows of the assignment pipeline, handled together (round 5) -------------------------------
// After a scheduling cycle places its pods, each placed pod p goes through six events at fixed offsets
// from its assignment time T_p = t + (cycle duration so far) + sched_to_as (the offsets are the network
// delays): AS_ASSIGN_REQ, PS_ASSIGN_REQ (+as_to_ps), AS_ASSIGN_RESP (+as_to_ps), N_BIND (+as_to_node),
// AS_POD_STARTED (+as_to_node), PS_POD_STARTED (+as_to_ps).  The pods of a cycle are 4 us apart, so in
// dslab order the six kinds interleave event by event: no two consecutive events share a kind (no run),
// yet within any as_to_ps-long stretch (50 ms at C3) they are independent.  A window is such a stretch:
// the next W events in dslab order, taken from the delay-class rings (their first 16 entries each, the
// first four rings of the source list), handled as W lanes at once.  The backlog regime adds a second
// pipeline of the same shape: a cycle's failed attempts are 4.1 ms apart (the per-node scheduling
// time) and each relays AS_POD_NOT_SCHEDULED -> PS_POD_NOT_SCHEDULED (+as_to_ps, no emission after
// that), so those two kinds are window kinds as well.
//
// Why it is exact.
// (1) The window is a prefix of dslab's order.  The rings' candidates are merged by (time, id), with
//     ranks by binary search.  The window stops before the first event that is not a candidate (a
//     later source's head, a ring's 16th entry, an event past the time limit) or not a window kind.
// (2) Nothing a window event emits can precede a later window event.  Every emission of these kinds
//     is at least min(as_to_ps, as_to_node) after its event (the finish of N_BIND adds the pod's
//     duration >= 0), every window event is at most that far after the first one, and an emission
//     at an equal time has a larger id.
// (3) The handlers commute inside a window.  Each writes only:
//     * its own pod's line (two events of one pod never share a window);
//     * storage's copy of its node (PS_ASSIGN_REQ: two assignments to one node never share a
//       window) or its node component's slot (N_BIND: likewise per slot);
//     * commutative header counters (storage's unscheduled count as a sum of +1 / -1) and the
//       group's running count (an atomic add).
//     It reads nothing the others write.
// Emissions get the ids a serial run would hand out: next_seq plus the emission counts of the
// earlier window events, N_BIND's finish before its start.  They are appended to their rings in that
// order (one delay per ring: times stay sorted), and the finishes go into the event heap one by one.
// A reference panic of these handlers, a full ring or heap, the cluster autoscaler (storage's
// assignment lists) or signed event times end the window before the event (or refuse it); the
// serial path then handles that event.
// Measured and not kept: storage's and the scheduler's PodFinishedRunning as window kinds (+2.6 % at
// C3, +2.4 % on the backlog; profiles/r05_ab9_win_finish.json): at C3 those windows hold about two
// events, and the estimator's in-order update grew this function past the VGPRs the event loop
// leaves free across the call.
#define K10S_WIN_PER_SRC 16
struct WinEv {
    double time, x;
    uint32_t seq, kind, a, b, src;
    int32_t slot;
};
// What a window event's handler needs of the replica's state (loaded once, checked, then applied).
struct WinSt {
    uint32_t rc, pf, nf, nep, ncpu, srun, removed, sflags, emits;
    uint64_t rr, nram;
    int32_t as_slot, snode, prs, g;
    double dur;
    bool pending;
};
// Entry i (< count) of ring q as the event loop would see it (LDS window below wend, else HBM).
K10S_HD HeapEv win_ring_entry(Ctx& c, uint32_t q, uint32_t i) {
    const RepHdr& H = c.H();
    const uint32_t hd = H.fq[q].head, we = H.fq[q].wend, pos = hd + i;
    if (pos - hd < we - hd) return H.fq_win[q * K10S_FQW + (pos & (K10S_FQW - 1))];
    return c.V().fq()[q * c.Ly().cap_fq + (pos & (c.Ly().cap_fq - 1))];
}
K10S_HD WinSt win_load(Ctx& c, const WinEv& e) {
    WinSt s;
    s.rc = s.pf = s.nf = s.nep = s.ncpu = s.srun = s.removed = s.sflags = s.emits = 0;
    s.rr = s.nram = 0;
    s.as_slot = s.snode = s.prs = s.g = -1;
    s.dur = 0.0;
    s.pending = false;
    switch (e.kind) {
    case K10S_EV_AS_ASSIGN_REQ:   // api_server.rs:163-192
        s.as_slot = c.V().node(e.b).as_slot;
        s.pending = c.H().pend_rm_n != 0 && bit_test(c.V().pend_rm(), c.S().node_uid[e.b]);
        s.emits = (s.pending || s.as_slot < 0) ? 0u : 1u;
        break;
    case K10S_EV_PS_ASSIGN_REQ: {   // persistent_storage.rs:250-294
        const PodState& P = c.V().pod(e.a);
        const NodeState& N = c.V().node(e.b);
        s.pf = P.flags;
        s.rc = P.req_cpu;
        s.rr = P.req_ram;
        s.nf = N.flags;
        s.nep = N.ps_epoch;
        s.ncpu = N.ps_cpu;
        s.nram = N.ps_ram;
        s.emits = 1;
        break;
    }
    case K10S_EV_AS_ASSIGN_RESP:   // api_server.rs:194-217
        s.as_slot = c.V().node(e.b).as_slot;
        s.emits = 1;
        break;
    case K10S_EV_N_BIND: {   // node_component.rs:181-202, 114-175
        const SlotState& SL = c.V().slot(e.slot);
        const PodState& P = c.V().pod(e.a);
        s.removed = SL.removed;
        s.snode = SL.node;
        s.srun = (uint32_t)SL.running;
        s.prs = P.run_slot;
        s.dur = P.dur;
        s.rc = P.req_cpu;
        s.rr = P.req_ram;
        s.sflags = c.S().pod_flags[e.a];
        s.g = c.S().pod_group[e.a];
        s.emits = (s.sflags & POD_HAS_DUR) ? 2u : 1u;
        break;
    }
    case K10S_EV_AS_POD_STARTED:         // api_server.rs:233-245
    case K10S_EV_AS_POD_NOT_SCHEDULED:   // api_server.rs:219-231
        s.emits = 1;
        break;
    default:   // K10S_EV_PS_POD_STARTED (persistent_storage.rs:309-314), K10S_EV_PS_POD_NOT_SCHEDULED
               // (296-307): no emission
        s.pf = c.V().pod(e.a).flags;
        break;
    }
    return s;
}
// Would the serial handler panic (or do what the window does not model)?  Then the window ends here.
K10S_HD bool win_bad(Ctx& c, const WinEv& e, const WinSt& s) {
    switch (e.kind) {
    case K10S_EV_PS_ASSIGN_REQ: return !(s.pf & PF_IN_PS) || !(s.nf & NF_PS_PRESENT) || (s.nf & NF_CA_ORIGIN);
    case K10S_EV_AS_ASSIGN_RESP: return s.as_slot < 0;
    case K10S_EV_N_BIND: return s.removed != 0 || s.snode != (int32_t)e.b || s.prs >= 0;
    case K10S_EV_PS_POD_STARTED: return (!K10S_TIME_KEY_ID || c.H().ps_rm_n != 0) && !(s.pf & PF_IN_PS);
    case K10S_EV_PS_POD_NOT_SCHEDULED: return !(s.pf & PF_IN_PS);
    default: return false;
    }
}
// The state writes of one window event (its emissions are written by the caller).  fseq: the id of
// N_BIND's finish self-event.
K10S_HD void win_apply(Ctx& c, const WinEv& e, const WinSt& s, uint32_t fseq) {
    switch (e.kind) {
    case K10S_EV_PS_ASSIGN_REQ: {
        PodState& P = c.V().pod(e.a);
        NodeState& N = c.V().node(e.b);
        P.ps_assigned = (int32_t)e.b;
        if (s.pf & PF_UNSCHED) P.flags = (uint8_t)(s.pf & ~PF_UNSCHED);
        N.ps_cpu = s.ncpu - s.rc;
        N.ps_ram = s.nram - s.rr;
        P.ps_aepoch = s.nep;
        break;
    }
    case K10S_EV_N_BIND: {
        c.V().slot(e.slot).running = (int32_t)s.srun + 1;
        PodState& P = c.V().pod(e.a);
        P.run_slot = e.slot;
        P.finish_seq = fseq;
        if (c.Ly().cap_gauge) {
            c.V().g_cpu()[e.slot] -= s.rc;
            c.V().g_ram()[e.slot] -= s.rr;
        }
        if (s.g >= 0) {
#if K10S_DEVICE
            atomicAdd(&c.V().grp()[s.g].running, 1u);
#else
            c.V().grp()[s.g].running += 1;
#endif
        }
        break;
    }
    case K10S_EV_PS_POD_STARTED:
        if (c.V().prec()) c.V().prec()[e.a].t_running = e.x;
        break;
    case K10S_EV_PS_POD_NOT_SCHEDULED:   // (the unscheduled count is summed by the caller)
        if (!(s.pf & PF_UNSCHED)) c.V().pod(e.a).flags = (uint8_t)(s.pf | PF_UNSCHED);
        break;
    default:
        break;
    }
}
// The window event's change of storage's unscheduled-pod count.
K10S_HD int32_t win_unsched_delta(const WinEv& e, const WinSt& s) {
    if (e.kind == K10S_EV_PS_ASSIGN_REQ) return (s.pf & PF_UNSCHED) ? -1 : 0;
    if (e.kind == K10S_EV_PS_POD_NOT_SCHEDULED) return (s.pf & PF_UNSCHED) ? 0 : 1;
    return 0;
}
// The ring emission of a window event (AS_TO_PS or AS_TO_NODE class), id seq.
K10S_HD HeapEv win_ring_emission(const Params& pr, const WinEv& e, uint32_t seq) {
    HeapEv o;
    o.seq = seq;
    o.slot = -1;
    o.a = e.a;
    o.b = 0;
    o.x = 0.0;
    switch (e.kind) {
    case K10S_EV_AS_ASSIGN_REQ:
        o.kind = K10S_EV_PS_ASSIGN_REQ, o.time = e.time + pr.as_to_ps_network_delay, o.b = e.b, o.x = e.x;
        break;
    case K10S_EV_PS_ASSIGN_REQ:
        o.kind = K10S_EV_AS_ASSIGN_RESP, o.time = e.time + pr.as_to_ps_network_delay, o.b = e.b;
        break;
    case K10S_EV_AS_ASSIGN_RESP:   // the slot found by win_load is the event's (e.slot is set by the caller)
        o.kind = K10S_EV_N_BIND, o.time = e.time + pr.as_to_node_network_delay, o.b = e.b, o.slot = e.slot;
        break;
    case K10S_EV_N_BIND:
        o.kind = K10S_EV_AS_POD_STARTED, o.time = e.time + pr.as_to_node_network_delay, o.x = e.time;
        break;
    case K10S_EV_AS_POD_NOT_SCHEDULED:
        o.kind = K10S_EV_PS_POD_NOT_SCHEDULED, o.time = e.time + pr.as_to_ps_network_delay, o.x = e.x;
        break;
    default:   // K10S_EV_AS_POD_STARTED
        o.kind = K10S_EV_PS_POD_STARTED, o.time = e.time + pr.as_to_ps_network_delay, o.x = e.x;
        break;
    }
    return o;
}
K10S_HD uint32_t win_ring_of(uint32_t kind) {   // the emission's delay class (N_BIND: its start)
    return (kind == K10S_EV_AS_ASSIGN_RESP || kind == K10S_EV_N_BIND) ? (uint32_t)FQ_AS_TO_NODE : (uint32_t)FQ_AS_TO_PS;
}
// One event into the dslab heap (emit's heap path with a given id; capacity checked by the caller).
K10S_HD void heap_insert(Ctx& c, const HeapEv& e) {
    RepHdr& H = c.H();
    const int64_t k = total_key(e.time);
    uint32_t pos = uniform_u32(H.heap_size);
    H.heap_size = pos + 1;
    [[maybe_unused]] uint32_t it = 0;
    while (pos > 0) {
        if (K10S_LOOP_CAP(it, 12, XG_LOOP_EMIT)) break;
        const uint32_t parent = (pos - 1) / K10S_HEAP_D;
        HeapEv p = heap_get(c, parent);
        uniform_event(p);
        const int64_t kp = total_key(p.time);
        if (!(k < kp || (k == kp && e.seq < p.seq))) break;
        heap_put(c, pos, p);
        pos = parent;
    }
    heap_put(c, pos, e);
    if (pos == 0) {
        H.heap_top = e;
        sl_mark(H, SRC_HEAP);
    }
}

// Called by the handler entry of the current event (a window kind at the head of ring sl[0].src; the
// clock is its time): handle the window it starts (W >= 2 events) and return W, or 0 (nothing written).
// Like run_batch, events 1..W-1 are logged and counted here, the rings are advanced past every window
// event except the current one (the event loop's consume removes it) and every ring touched is marked
// for the source list.
K10S_HD_NOINL uint32_t win_batch(Ctx& c) {
    RepHdr& H = c.H();
    [[maybe_unused]] const uint64_t t_front = prof_now();
    const uint32_t fl = uniform_u32(H.run_flags);
    if (!(fl & 1u) || (!(fl & 2u) && (int64_t)uniform_u64((uint64_t)H.pods_left) <= 0)) return 0;
    if (!c.Ly().tnonneg || c.S().ca_enabled || !c.Ly().cap_fq) return 0;
    const uint32_t src0 = uniform_u32(H.sl[0].src);
    if (src0 >= (uint32_t)K10S_NFQ) return 0;
    const Params& pr = c.P();
    const double t0 = uniform_f64(H.clock), lim = uniform_f64(H.run_limit);
    const double d_ps = pr.as_to_ps_network_delay, d_node = pr.as_to_node_network_delay;
    const double tlook = t0 + (d_ps < d_node ? d_ps : d_node);
    const int64_t kmax = total_key(tlook < lim ? tlook : lim);   // a candidate's time is at most this
    // the first (up to) four rings of the source list; the first other source bounds the window
    const uint32_t sn = uniform_u32(H.sl_n);
    uint32_t srcs[4] = {0u, 0u, 0u, 0u};
    uint32_t m = 0;
    int64_t bk = 0x7FFFFFFFFFFFFFFFll;
    uint32_t bs = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < sn; i++) {
        const uint32_t s = uniform_u32(H.sl[i].src);
        if (s < (uint32_t)K10S_NFQ && m < 4) {
            if (m == 0) srcs[0] = s;
            else if (m == 1) srcs[1] = s;
            else if (m == 2) srcs[2] = s;
            else srcs[3] = s;
            m++;
            continue;
        }
        bk = (int64_t)uniform_u64((uint64_t)H.sl[i].key);
        bs = uniform_u32(H.sl[i].seq);
        break;
    }
    // a ring holding more than K10S_WIN_PER_SRC entries: its 16th bounds the window (only 15 are used)
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t q = j == 0 ? srcs[0] : j == 1 ? srcs[1] : j == 2 ? srcs[2] : srcs[3];
        if (uniform_u32(H.fq[q].tail - H.fq[q].head) > K10S_WIN_PER_SRC) {
            const HeapEv b = win_ring_entry(c, q, K10S_WIN_PER_SRC - 1);
            const int64_t kb = (int64_t)uniform_u64((uint64_t)total_key(b.time));
            const uint32_t sb = uniform_u32(b.seq);
            if (sl_less(kb, sb, bk, bs)) bk = kb, bs = sb;
        }
    }
    uint32_t W = 0, V = 0;
#if K10S_DEVICE
    // ---- candidates: lane 16j + i holds entry i of ring srcs[j]
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t grp = lane >> 4, gi = lane & 15u;
    const uint32_t myq = grp == 0 ? srcs[0] : grp == 1 ? srcs[1] : grp == 2 ? srcs[2] : srcs[3];
    WinEv ev;
    ev.time = 0.0;
    ev.x = 0.0;
    ev.seq = 0xFFFFFFFFu;
    ev.kind = 0xFFFFu;
    ev.a = ev.b = 0;
    ev.slot = -1;
    ev.src = myq;
    int64_t key = 0x7FFFFFFFFFFFFFFFll;
    bool valid = false;
    if (grp < m && gi < H.fq[myq].tail - H.fq[myq].head) {
        const HeapEv h = win_ring_entry(c, myq, gi);
        ev.time = h.time;
        ev.x = h.x;
        ev.seq = h.seq;
        ev.kind = h.kind;
        ev.slot = h.slot;
        ev.a = h.a;
        ev.b = h.b;
        key = total_key(h.time);
        valid = key <= kmax && sl_less(key, ev.seq, bk, bs);
    }
    // (the valid entries of a ring are a prefix of its 16: keys increase along a ring)
    const uint64_t vm = __ballot(valid);
    V = (uint32_t)__popcll(vm);
    if (V < 2) return 0;
    // ---- rank = position in the merged (time, id) order: own index + the other rings' entries below
    uint32_t rank = gi;
    const uint32_t klo = (uint32_t)(uint64_t)key, khi = (uint32_t)((uint64_t)key >> 32);
    K10S_UNROLL
    for (uint32_t j = 0; j < 4; j++) {
        if (j >= m) break;
        const uint32_t vj = (uint32_t)__popcll((vm >> (16u * j)) & 0xFFFFull);
        uint32_t lo = 0, hi = grp == j ? 0u : vj;
        K10S_UNROLL
        for (int step = 0; step < 5; step++) {   // binary search over <= 16 sorted entries
            const uint32_t mid = (lo + hi) >> 1;
            const int addr = (int)((16u * j + (mid < 15u ? mid : 15u)) * 4u);
            const uint32_t xl = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)klo);
            const uint32_t xh = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)khi);
            const uint32_t xs = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)ev.seq);
            const bool less = lo < hi && sl_less((int64_t)(((uint64_t)xh << 32) | xl), xs, key, ev.seq);
            const bool go = lo < hi;
            lo = go && less ? mid + 1u : lo;
            hi = go && !less ? mid : hi;
        }
        rank += lo;
    }
    {   // invalid lanes take the ranks after V, in lane order
        const uint32_t below = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(vm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)vm, 0u));
        if (!valid) rank = V + (lane - below);
    }
    // ---- lanes into (time, id) order: lane r holds the window's r-th event
    {
        const int addr = (int)(rank * 4u);
        auto mv = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)v); };
        const uint64_t tb = f2u(ev.time), xb = f2u(ev.x);
        const uint32_t t_lo = mv((uint32_t)tb), t_hi = mv((uint32_t)(tb >> 32));
        const uint32_t x_lo = mv((uint32_t)xb), x_hi = mv((uint32_t)(xb >> 32));
        ev.seq = mv(ev.seq);
        const uint32_t ks = mv(ev.kind | ((uint32_t)(uint16_t)ev.slot << 16));
        ev.a = mv(ev.a);
        ev.b = mv(ev.b);
        ev.src = mv(ev.src);
        ev.time = u2f(((uint64_t)t_hi << 32) | t_lo);
        ev.x = u2f(((uint64_t)x_hi << 32) | x_lo);
        ev.kind = ks & 0xFFFFu;
        ev.slot = (int32_t)(int16_t)(ks >> 16);
    }
    const uint32_t r = lane;
    const bool live = r < V;
    const bool wk = live && ((K10S_WIN_KINDS >> (ev.kind & 63u)) & 1ull) != 0 && ev.kind < 64u;
    WinSt st;
    st.rc = st.pf = st.nf = st.nep = st.ncpu = st.srun = st.removed = st.sflags = st.emits = 0;
    st.rr = st.nram = 0;
    st.as_slot = st.snode = st.prs = st.g = -1;
    st.dur = 0.0;
    st.pending = false;
    if (wk) st = win_load(c, ev);   // (only window events: another kind's fields index other tables)
    if (wk && ev.kind == K10S_EV_AS_ASSIGN_RESP) ev.slot = st.as_slot;   // N_BIND's component
    bool stop = !wk || win_bad(c, ev, st);
    // two events of one pod, two assignments to one node, two binds on one component: only the first
    {
        const uint32_t writer = wk && (ev.kind == K10S_EV_PS_ASSIGN_REQ || ev.kind == K10S_EV_N_BIND ||
                                       ev.kind == K10S_EV_PS_POD_STARTED || ev.kind == K10S_EV_PS_POD_NOT_SCHEDULED) ? 1u : 0u;
        uint64_t wm = __ballot(writer != 0u) & (V >= 64u ? ~0ull : ((1ull << V) - 1ull));
        while (wm) {
            const uint32_t b = (uint32_t)__builtin_ctzll(wm);
            wm &= wm - 1;
            const uint32_t bk2 = (uint32_t)__builtin_amdgcn_readlane((int)ev.kind, (int)b);
            const uint32_t ba = (uint32_t)__builtin_amdgcn_readlane((int)ev.a, (int)b);
            const uint32_t bb = (uint32_t)__builtin_amdgcn_readlane((int)ev.b, (int)b);
            const int32_t bsl = __builtin_amdgcn_readlane(ev.slot, (int)b);
            stop |= r > b && (ev.a == ba || (ev.kind == bk2 && ((bk2 == K10S_EV_PS_ASSIGN_REQ && ev.b == bb) ||
                                                                 (bk2 == K10S_EV_N_BIND && ev.slot == bsl))));
        }
    }
    {
        const uint64_t sm = __ballot(stop);
        W = sm ? (uint32_t)__builtin_ctzll(sm) : 64u;
    }
    W = uniform_u32(W);
    K10S_PROF_ADD(c, PROF_WFRONT, t_front);
    if (W < 2) return 0;
    const bool in = r < W;
    // ---- emissions: ids and ring positions in window order
    const uint32_t ne = in ? st.emits : 0u;
    const bool e_heap = in && ev.kind == K10S_EV_N_BIND && (st.sflags & POD_HAS_DUR);
    const bool e_ring = ne > (e_heap ? 1u : 0u);
    const uint32_t e_q = win_ring_of(ev.kind);
    const bool e_ps = e_ring && e_q == (uint32_t)FQ_AS_TO_PS, e_node = e_ring && e_q == (uint32_t)FQ_AS_TO_NODE;
    const uint64_t m1 = __ballot(ne >= 1u), m2 = __ballot(ne >= 2u), mps = __ballot(e_ps), mnd = __ballot(e_node);
    const uint64_t mhp = __ballot(e_heap);
    auto below = [&](uint64_t mk) {
        return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
    };
    const uint32_t n_total = (uint32_t)__popcll(m1) + (uint32_t)__popcll(m2);
    const uint32_t n_ps = (uint32_t)__popcll(mps), n_node = (uint32_t)__popcll(mnd), n_heap = (uint32_t)__popcll(mhp);
    const uint32_t id0 = uniform_u32(H.next_seq) + below(m1) + below(m2);
    // events consumed per ring (room for emissions into a ring that is also consumed)
    uint32_t used[4];
    K10S_UNROLL
    for (uint32_t j = 0; j < 4; j++) used[j] = j < m ? (uint32_t)__popcll(__ballot(in && ev.src == (j == 0 ? srcs[0] : j == 1 ? srcs[1] : j == 2 ? srcs[2] : srcs[3]))) : 0u;
#else
    // ---- host: the merge of the rings, event by event
    WinEv evs[64];
    WinSt sts[64];
    {
        uint32_t cur[4] = {0u, 0u, 0u, 0u};
        while (V < 64) {
            int best = -1;
            int64_t kbest = 0;
            uint32_t sbest = 0;
            HeapEv hb{};
            for (uint32_t j = 0; j < m; j++) {
                const uint32_t q = srcs[j];
                if (cur[j] >= K10S_WIN_PER_SRC || cur[j] >= H.fq[q].tail - H.fq[q].head) continue;
                const HeapEv h = win_ring_entry(c, q, cur[j]);
                const int64_t kh = total_key(h.time);
                if (best < 0 || sl_less(kh, h.seq, kbest, sbest)) best = (int)j, kbest = kh, sbest = h.seq, hb = h;
            }
            if (best < 0 || kbest > kmax || !sl_less(kbest, sbest, bk, bs)) break;
            cur[best]++;
            WinEv& e = evs[V++];
            e.time = hb.time;
            e.x = hb.x;
            e.seq = hb.seq;
            e.kind = hb.kind;
            e.slot = hb.slot;
            e.a = hb.a;
            e.b = hb.b;
            e.src = srcs[best];
        }
    }
    if (V < 2) return 0;
    for (W = 0; W < V; W++) {
        WinEv& e = evs[W];
        if (!((K10S_WIN_KINDS >> (e.kind & 63u)) & 1ull) || e.kind >= 64u) break;
        sts[W] = win_load(c, e);
        if (e.kind == K10S_EV_AS_ASSIGN_RESP) e.slot = sts[W].as_slot;
        if (win_bad(c, e, sts[W])) break;
        bool conf = false;
        for (uint32_t b = 0; b < W; b++) {
            const WinEv& o = evs[b];
            const bool writer = o.kind == K10S_EV_PS_ASSIGN_REQ || o.kind == K10S_EV_N_BIND || o.kind == K10S_EV_PS_POD_STARTED ||
                                o.kind == K10S_EV_PS_POD_NOT_SCHEDULED;
            conf |= writer && (e.a == o.a || (e.kind == o.kind && ((o.kind == K10S_EV_PS_ASSIGN_REQ && e.b == o.b) ||
                                                                     (o.kind == K10S_EV_N_BIND && e.slot == o.slot))));
        }
        if (conf) break;
    }
    if (W < 2) return 0;
    uint32_t n_total = 0, n_ps = 0, n_node = 0, n_heap = 0;
    uint32_t used[4] = {0u, 0u, 0u, 0u};
    for (uint32_t r = 0; r < W; r++) {
        const WinSt& s = sts[r];
        const bool hp = evs[r].kind == K10S_EV_N_BIND && (s.sflags & POD_HAS_DUR);
        n_total += s.emits;
        n_heap += hp ? 1u : 0u;
        if (s.emits > (hp ? 1u : 0u)) {
            if (win_ring_of(evs[r].kind) == (uint32_t)FQ_AS_TO_PS) n_ps++;
            else n_node++;
        }
        for (uint32_t j = 0; j < m; j++) used[j] += evs[r].src == srcs[j] ? 1u : 0u;
    }
#endif
    // ---- what the serial path would place differently: then no window
    [[maybe_unused]] const uint64_t t_apply = prof_now();
    const uint32_t seq0 = uniform_u32(H.next_seq);
    if ((uint64_t)seq0 + n_total > 0xFFFFFFFFull) return 0;
    if (n_heap && uniform_u32(H.heap_size) + n_heap > c.Ly().cap_heap) return 0;
    const uint32_t cap = c.Ly().cap_fq;
    uint32_t rhd[2], rtl[2], rwe[2];
    for (uint32_t z = 0; z < 2; z++) {
        const uint32_t q = z == 0 ? (uint32_t)FQ_AS_TO_PS : (uint32_t)FQ_AS_TO_NODE;
        const uint32_t n = z == 0 ? n_ps : n_node;
        rhd[z] = uniform_u32(H.fq[q].head);
        rtl[z] = uniform_u32(H.fq[q].tail);
        rwe[z] = uniform_u32(H.fq[q].wend);
        if (!n) continue;
        uint32_t consumed = 0;
        for (uint32_t j = 0; j < m; j++) consumed += (j == 0 ? srcs[0] : j == 1 ? srcs[1] : j == 2 ? srcs[2] : srcs[3]) == q ? used[j] : 0u;
        if (cap - (rtl[z] - rhd[z]) + consumed < n) return 0;
        // the ring stays sorted: its first new entry is not before its newest one
        const double d = z == 0 ? d_ps : d_node;
        if (rtl[z] != rhd[z] && total_key(t0 + d) < total_key(uniform_f64(H.fq[q].last))) return 0;
    }
    const uint32_t cap_log = c.Ly().cap_log;
    const uint32_t log0 = uniform_u32(H.log_n) - 1u;   // event 0 was logged by the event loop
    double last_ps = 0.0, last_node = 0.0, tW = t0;
    uint32_t unsched = 0;
#if K10S_DEVICE
    {
        const uint32_t fseq = e_heap ? id0 : 0u;   // N_BIND: its finish first (id0), then its start
        if (in) {
            win_apply(c, ev, st, fseq);
            unsched = (uint32_t)win_unsched_delta(ev, st);
            if (cap_log && r > 0 && log0 + r < cap_log) {
                k10s_log_entry le;
                le.time = ev.time;
                le.seq = ev.seq;
                le.kind = (uint16_t)ev.kind;
                le.slot = (int16_t)(ev.kind == K10S_EV_N_BIND ? ev.slot : -1);
                le.pod = (int32_t)ev.a;
                le.node = (ev.kind == K10S_EV_AS_POD_STARTED || ev.kind == K10S_EV_PS_POD_STARTED ||
                           ev.kind == K10S_EV_AS_POD_NOT_SCHEDULED || ev.kind == K10S_EV_PS_POD_NOT_SCHEDULED) ? -1 : (int32_t)ev.b;
                c.V().log()[log0 + r] = le;
            }
        }
        if (e_ring) {
            const uint32_t z = e_ps ? 0u : 1u;
            const uint32_t q = e_ps ? (uint32_t)FQ_AS_TO_PS : (uint32_t)FQ_AS_TO_NODE;
            const uint32_t idx = e_ps ? below(mps) : below(mnd);
            const uint32_t tl = z == 0 ? rtl[0] : rtl[1], hd = z == 0 ? rhd[0] : rhd[1], we = z == 0 ? rwe[0] : rwe[1];
            const HeapEv o = win_ring_emission(pr, ev, id0 + (e_heap ? 1u : 0u));
            c.V().fq()[q * cap + ((tl + idx) & (cap - 1))] = o;
            if (we == tl && (tl - hd) + idx < K10S_FQW) H.fq_win[q * K10S_FQW + ((tl + idx) & (K10S_FQW - 1))] = o;
        }
        // the rings' newest times and the last event's time (lane readlanes of the last writers)
        if (n_ps) last_ps = uniform_f64(__shfl(ev.time, 63 - (int)__builtin_clzll(mps))) + d_ps;
        if (n_node) last_node = uniform_f64(__shfl(ev.time, 63 - (int)__builtin_clzll(mnd))) + d_node;
        tW = uniform_f64(__shfl(ev.time, (int)W - 1));
        // the finishes into the heap, one by one in window order
        uint64_t hm = mhp;
        while (hm) {
            const uint32_t b = (uint32_t)__builtin_ctzll(hm);
            hm &= hm - 1;
            HeapEv f;
            f.time = uniform_f64(__shfl(ev.time + (st.dur + d_node), (int)b));   // clock + delay, as emit
            f.seq = uniform_u32((uint32_t)__builtin_amdgcn_readlane((int)id0, (int)b));
            f.kind = (uint16_t)K10S_EV_N_POD_FINISHED;
            f.slot = (int16_t)__builtin_amdgcn_readlane(ev.slot, (int)b);
            f.a = uniform_u32((uint32_t)__builtin_amdgcn_readlane((int)ev.a, (int)b));
            f.b = uniform_u32((uint32_t)__builtin_amdgcn_readlane((int)ev.b, (int)b));
            f.x = uniform_f64(__shfl(ev.time + st.dur, (int)b));
            heap_insert(c, f);
        }
    }
    unsched = wave_sum_u32(unsched);
#else
    {
        uint32_t id = seq0, ips = 0, ind = 0;
        for (uint32_t r = 0; r < W; r++) {
            const WinEv& e = evs[r];
            const WinSt& s = sts[r];
            const bool hp = e.kind == K10S_EV_N_BIND && (s.sflags & POD_HAS_DUR);
            win_apply(c, e, s, hp ? id : 0u);
            unsched += (uint32_t)win_unsched_delta(e, s);
            if (cap_log && r > 0 && log0 + r < cap_log) {
                k10s_log_entry le;
                le.time = e.time;
                le.seq = e.seq;
                le.kind = (uint16_t)e.kind;
                le.slot = (int16_t)(e.kind == K10S_EV_N_BIND ? e.slot : -1);
                le.pod = (int32_t)e.a;
                le.node = (e.kind == K10S_EV_AS_POD_STARTED || e.kind == K10S_EV_PS_POD_STARTED ||
                           e.kind == K10S_EV_AS_POD_NOT_SCHEDULED || e.kind == K10S_EV_PS_POD_NOT_SCHEDULED) ? -1 : (int32_t)e.b;
                c.V().log()[log0 + r] = le;
            }
            if (hp) {
                HeapEv f;
                f.time = e.time + (s.dur + d_node);   // clock + delay, as emit
                f.seq = id;
                f.kind = (uint16_t)K10S_EV_N_POD_FINISHED;
                f.slot = (int16_t)e.slot;
                f.a = e.a;
                f.b = e.b;
                f.x = e.time + s.dur;
                heap_insert(c, f);
            }
            const bool ring = s.emits > (hp ? 1u : 0u);
            if (ring) {
                const bool ps = win_ring_of(e.kind) == (uint32_t)FQ_AS_TO_PS;
                const uint32_t z = ps ? 0u : 1u, q = ps ? (uint32_t)FQ_AS_TO_PS : (uint32_t)FQ_AS_TO_NODE;
                const uint32_t idx = ps ? ips++ : ind++;
                const HeapEv o = win_ring_emission(pr, e, id + (hp ? 1u : 0u));
                c.V().fq()[q * cap + ((rtl[z] + idx) & (cap - 1))] = o;
                if (rwe[z] == rtl[z] && (rtl[z] - rhd[z]) + idx < K10S_FQW)
                    H.fq_win[q * K10S_FQW + ((rtl[z] + idx) & (K10S_FQW - 1))] = o;
                if (ps) last_ps = o.time;
                else last_node = o.time;
            }
            id += s.emits;
        }
        tW = evs[W - 1].time;
    }
#endif
    wave_sync();
    // ---- header: logs, counters, rings, ids, clock
    if (cap_log) {   // (the loop logged event 0 at log0, or flagged the overflow)
        if (log0 + W <= cap_log) H.log_n = log0 + W;
        else {
            H.log_n = log0 + 1u < cap_log ? cap_log : log0 + 1u;
            H.flags |= 1u;
        }
    }
    H.unsched_cache_count += unsched;   // (a wrapping sum of the events' +1 / -1)
    for (uint32_t z = 0; z < 2; z++) {
        const uint32_t n = z == 0 ? n_ps : n_node;
        if (!n) continue;
        const uint32_t q = z == 0 ? (uint32_t)FQ_AS_TO_PS : (uint32_t)FQ_AS_TO_NODE;
        if (rwe[z] == rtl[z] && rtl[z] - rhd[z] < K10S_FQW) {
            const uint32_t room = K10S_FQW - (rtl[z] - rhd[z]);
            H.fq[q].wend = rtl[z] + (n < room ? n : room);
        }
        H.fq[q].tail = rtl[z] + n;
        H.fq[q].last = z == 0 ? last_ps : last_node;
        sl_mark(H, q);
    }
    H.next_seq = seq0 + n_total;
    H.clock = tW;
    H.counters[K10S_C_EVENTS] += W - 1u;
    // ---- advance the rings past the window's events (the current one stays for the loop's consume)
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t q = j == 0 ? srcs[0] : j == 1 ? srcs[1] : j == 2 ? srcs[2] : srcs[3];
        const uint32_t n = used[j] - (q == src0 ? 1u : 0u);
        if (!n) continue;
        const uint32_t hd = uniform_u32(H.fq[q].head) + n, tl = uniform_u32(H.fq[q].tail), we = uniform_u32(H.fq[q].wend);
        H.fq[q].head = hd;
        if ((int32_t)(hd - we) >= 0) {
            if (hd != tl) fq_refill(c, (int)q, hd);
            else H.fq[q].wend = hd;
        }
        if (q != src0) sl_mark(H, q);
    }
#if !K10S_DEVICE && defined(K10S_HOST_STATS)
    k10s_host_stats[HS_WINDOWS] += 1;
    k10s_host_stats[HS_WIN_EVENTS] += W;
    k10s_host_stats[HS_EVENTS] += W - 1;
#endif
    K10S_PROF_ADD(c, PROF_WAPPLY, t_apply);
    return W;
}

// Returns 1 if the replica still has work (event budget exhausted), else 0.  The working header
// c.H() is LDS on the device (staged by the kernel) and the replica's header in place on the host.
K10S_HD int run_replica(Ctx& c, int mode, double until_time, double max_time, uint64_t budget) {
    RepHdr* h = &c.H();
    if (h->status != K10S_REPLICA_RUNNING) return 0;
    h->cur_kind = 0xFFFF;
    h->cur_seq = 0;
    // launch constants are re-read at each use (scalar loads through the opaque constant pointer)
    // rather than held in SGPRs across the loop, where they are spilled around the handler calls
#define ntr (c.S().n_trace)
#define cap_log (c.Ly().cap_log)
    // one time limit per mode (until_time / max_time)
    const uint32_t until_mode0 = mode == K10S_RUN_UNTIL_TIME ? 1u : 0u;
    const double limit = until_mode0 ? until_time : max_time;
    auto until_mode = [&]() -> bool { return until_mode0 != 0; };
    uint64_t done = 0;
    int more = 0;
    uint32_t status = K10S_REPLICA_RUNNING;
    const uint64_t t_loop = prof_now();
    sl_rebuild(c, ntr);  // the sorted source list, from the sources' heads
    h->run_flags = (budget == 0 ? 1u : 0u) | (until_mode0 ? 2u : 0u);   // run_batch, win_batch
#if !K10S_DEVICE && defined(K10S_TRAFFIC_MODEL)
    k10s_tm_replica(c.V().b, &c.Ly());
#endif
    h->run_limit = limit;
    [[maybe_unused]] uint32_t it_stale = 0;
#if !K10S_DEVICE && defined(K10S_HOST_STATS)
    uint32_t hs_next_before = 0xFFFFFFFFu;
#endif
    while (!h->error_code) {
        if (!until_mode() && h->pods_left <= 0 && is_multiple_of_1000(h->clock)) {
            status = K10S_REPLICA_FINISHED;
            break;
        }
        // next non-canceled event: the head of the first source in the source list (the minimum
        // (time, id) over the shared trace stream, the heap root and the delay-class FIFO heads)
        HeapEv e;
        int src = 0;
        bool have = false;
        const uint64_t t_sel = prof_now();
        sl_apply_dirty(c, ntr);
        EvRef ep = K10S_EVREF(&h->heap_top);
        for (;;) {
            if (uniform_u32(h->sl_n) == 0) break;
            src = (int)uniform_u32(h->sl[0].src);
            if (src == SRC_TRACE) {
                const uint32_t cur = h->trace_cursor;
                const uint32_t tk = c.S().trace[cur].kind, ta = c.S().trace[cur].arg;
                e.time = c.S().trace[cur].time;
                e.seq = h->tr_seq;   // the replica's id (k10s_replica_params.workload_prefix)
                e.kind = (uint16_t)tk;
                e.slot = -1;
                e.x = 0.0;
                e.a = ta;
                e.b = 0;
                if (tk == K10S_EV_AS_CREATE_NODE_REQ) {
                    e.a = c.S().def_node[ta];
                    e.b = ta;
                }
                uniform_event(e);
                h->cur_ev = e;
                ep = K10S_EVREF(&h->cur_ev);
            } else if (src == SRC_HEAP) {
                e.kind = (uint16_t)uniform_u32(h->heap_top.kind);
                e.a = uniform_u32(h->heap_top.a);
                e.seq = uniform_u32(h->heap_top.seq);
                e.time = uniform_f64(h->heap_top.time);
                // canceled (lazy cancel): only while some canceled finish is pending is the pod read
                if (e.kind == K10S_EV_N_POD_FINISHED && uniform_u32(h->stale_fin) != 0 &&
                    uniform_u32(c.V().pod(e.a).finish_seq) != e.seq) {
                    drop_stale_head(c, ntr);
                    if (K10S_LOOP_CAP(it_stale, 1u << 24, XG_LOOP_STALE)) break;
                    continue;
                }
                ep = K10S_EVREF(&h->heap_top);
            } else {
                ep = K10S_EVREF(&h->fq_win[(uint32_t)src * K10S_FQW + (uniform_u32(h->fq[src].head) & (K10S_FQW - 1))]);
                e.time = uniform_f64(ep->time);
                e.seq = uniform_u32(ep->seq);
                e.kind = (uint16_t)uniform_u32(ep->kind);
            }
            have = true;
            break;
        }
        K10S_PROF_ADD(c, PROF_SELECT, t_sel);
        if (!have) {
            if (until_mode()) h->clock = limit;
            status = until_mode() ? K10S_REPLICA_RUNNING : K10S_REPLICA_FINISHED;
            break;
        }
        if (e.time > limit) {
            if (until_mode()) h->clock = limit;                // step_until_time: stop at the time
            else status = K10S_REPLICA_TIME_LIMIT;             // run until finished: max_time reached
            break;
        }
        if (budget && done >= budget) {
            more = 1;
            break;
        }
#if !K10S_DEVICE && defined(K10S_HOST_STATS)
        if (e.seq >= hs_next_before) {   // emitted by the previous event's handler
            K10S_HSTAT(HS_NEXT_EMITTED);
            if (src < K10S_NFQ) K10S_HSTAT(HS_NEXT_EMITTED_FIFO);
        }
        hs_next_before = h->next_seq;
#endif
        h->clock = e.time;
        h->cur_kind = e.kind;
        h->cur_seq = e.seq;
        fair_priority(done);
        done++;  // counters[K10S_C_EVENTS] takes the launch's count once, at exit (no per-event LDS RMW)
        if (cap_log) {
            e = *ep;   // parity logging: the whole event
            uniform_event(e);
            uint32_t k = h->log_n;
            if (k < cap_log) {
                k10s_log_entry le;
                le.time = e.time;
                le.seq = e.seq;
                le.kind = e.kind;
                le.slot = e.slot;
                int32_t pod = -1, node = -1;
                switch (e.kind) {
                case K10S_EV_AS_CREATE_NODE_REQ: case K10S_EV_AS_CREATE_NODE_RESP: case K10S_EV_AS_REMOVE_NODE_REQ:
                case K10S_EV_AS_REMOVE_NODE_RESP: case K10S_EV_AS_NODE_REMOVED: case K10S_EV_PS_CREATE_NODE_REQ:
                case K10S_EV_PS_NODE_ADDED: case K10S_EV_PS_REMOVE_NODE_REQ: case K10S_EV_PS_NODE_REMOVED:
                case K10S_EV_S_ADD_NODE: case K10S_EV_S_REMOVE_NODE: case K10S_EV_N_REMOVE_NODE:
                    node = (int32_t)e.a;
                    break;
                case K10S_EV_AS_ASSIGN_REQ: case K10S_EV_AS_ASSIGN_RESP: case K10S_EV_AS_POD_FINISHED:
                case K10S_EV_PS_ASSIGN_REQ: case K10S_EV_PS_POD_FINISHED: case K10S_EV_S_POD_FINISHED:
                case K10S_EV_N_BIND: case K10S_EV_N_POD_FINISHED:
                    pod = (int32_t)e.a;
                    node = (int32_t)e.b;
                    break;
                case K10S_EV_AS_REMOVE_POD_RESP:
                    pod = (int32_t)e.a;
                    node = f2u(e.x) ? (int32_t)e.b : -1;
                    break;
                case K10S_EV_AS_CREATE_POD_REQ: case K10S_EV_AS_POD_NOT_SCHEDULED: case K10S_EV_AS_POD_STARTED:
                case K10S_EV_AS_REMOVE_POD_REQ: case K10S_EV_AS_POD_REMOVED: case K10S_EV_PS_CREATE_POD_REQ:
                case K10S_EV_PS_POD_NOT_SCHEDULED: case K10S_EV_PS_POD_STARTED: case K10S_EV_PS_REMOVE_POD_REQ:
                case K10S_EV_PS_POD_REMOVED: case K10S_EV_S_POD_SCHEDULE_REQ: case K10S_EV_S_REMOVE_POD:
                case K10S_EV_N_REMOVE_POD:
                    pod = (int32_t)e.a;
                    break;
                default:
                    break;
                }
                le.pod = pod;
                le.node = node;
                c.V().log()[k] = le;
                h->log_n = k + 1;
            } else {
                h->flags |= 1u;
            }
        }
#if K10S_DEVICE && K10S_BEACON
        if (lane_id() == 0) {
            uint32_t* b = k10s_beacon + (uint64_t)blockIdx.x * K10S_BEACON_WORDS;
            const uint32_t w[12] = {(uint32_t)done, e.kind, e.seq, (uint32_t)f2u(e.time), (uint32_t)(f2u(e.time) >> 32),
                                    h->heap_size, h->stale_fin, h->sl_n, (uint32_t)src, h->aq_size, h->uq_size, e.a};
            for (int i = 11; i >= 0; i--)   // word 0 (the event count) last
                __hip_atomic_store(b + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#endif
        const uint64_t t_dis = prof_now();
        K10S_TM_EVENT(e.kind);
        dispatch(c, ep, e.kind);
        {   // the event stayed at the head of its source during the handler (an emission lands after
            // it: larger id, time >= clock); remove it now
            const uint64_t t_con = prof_now();
            consume_source(c, src, ntr);
            K10S_PROF_ADD(c, PROF_CONSUME, t_con);
        }
        K10S_PROF_ADD(c, PROF_DISPATCH, t_dis);
#if K10S_PROF
        h->prof[K10S_PROF_KIND0 + e.kind] += prof_now() - t_dis;
        h->prof[K10S_PROF_KIND0 + K10S_EV_NUM_KINDS + e.kind] += 1;
#endif
        if (e.kind == K10S_EV_M_GAUGE_TICK && c.Ly().stall && !until_mode() &&
            replica_stalled(c)) {
            status = K10S_REPLICA_STALLED;
            break;
        }
    }
    K10S_PROF_ADD(c, PROF_LOOP, t_loop);
    K10S_TM_EVENT(0xFFFFu);
#if K10S_DEVICE && K10S_BEACON
    if (lane_id() == 0)   // word 12: the loop has exited (1 + launch-local event count)
        __hip_atomic_store(k10s_beacon + (uint64_t)blockIdx.x * K10S_BEACON_WORDS + 12, (uint32_t)done + 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    h->counters[K10S_C_EVENTS] += done;
    if (h->error_code) status = K10S_REPLICA_ERROR;
    h->status = status;
    return more;
#undef ntr
#undef cap_log
}

}  // namespace k10s
