// TOOLING (tools/traffic_model.py): the runtime of the host engine's memory-touch model.  The engine
// (tests/hostcheck, built with -DK10S_TRAFFIC_MODEL and clang's -fsanitize-coverage=trace-loads,
// trace-stores) calls __sanitizer_cov_load*/store* before every load and store, k10s_tm_replica at
// each run of a replica and k10s_tm_event before each event's dispatch.  Every touched address inside
// the replica's region, outside its header (the header is LDS on the device), is attributed to its
// section (Layout) and to the kind of the event being handled: per event, the distinct 128-B lines
// read and the distinct 64-B chunks written ("cold": nothing survives between events), and the same
// through a per-replica LRU of TM_LRU_LINES lines ("warm": the replica's share of L2).
// This file is compiled without the tracing flags.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <list>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../kubernetriks_amd/csrc/k10s_state.h"

namespace {
constexpr int NK = 64;   // event kinds (K10S_EV_NUM_KINDS <= 64)
constexpr int NS = 48;   // sections
struct Sec {
    uint64_t off;
    std::string name;
};
struct St {
    const uint8_t* base = nullptr;
    uint64_t stride = 0, hdr_lo = 0, hdr_hi = 0;
    std::vector<Sec> secs;
    uint32_t kind = 0xFFFF;
    bool on = false;
    std::unordered_set<uint64_t> rd, wr;          // this event's lines / chunks (cold model)
    std::unordered_map<uint64_t, int> rd_sec, wr_sec;
    // warm model: LRU of lines
    std::list<uint64_t> lru;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> lru_pos;
    size_t lru_cap = 32;
    double cold_rd[NK][NS] = {}, cold_wr[NK][NS] = {}, warm_rd[NK][NS] = {}, raw_rd[NK][NS] = {};
    double events[NK] = {};
    bool in_hook = false;
} g;

int section_of(uint64_t off) {
    int s = -1;
    for (size_t i = 0; i < g.secs.size(); i++)
        if (g.secs[i].off <= off) s = (int)i;
    return s;
}
void touch(const void* p, bool write) {
    if (!g.on || g.in_hook) return;
    const uint8_t* a = (const uint8_t*)p;
    if (a < g.base || a >= g.base + g.stride) return;
    const uint64_t off = (uint64_t)(a - g.base);
    if (off >= g.hdr_lo && off < g.hdr_hi) return;
    g.in_hook = true;
    const int s = section_of(off);
    if (!write && g.kind < NK && s >= 0 && s < NS) g.raw_rd[g.kind][s] += 1;
    if (write) {
        const uint64_t ch = (uint64_t)(uintptr_t)a >> 6;
        if (g.wr.insert(ch).second) g.wr_sec[ch] = s;
    } else {
        const uint64_t ln = (uint64_t)(uintptr_t)a >> 7;
        if (g.rd.insert(ln).second) {
            g.rd_sec[ln] = s;
            auto it = g.lru_pos.find(ln);
            if (it != g.lru_pos.end()) {
                g.lru.erase(it->second);
            } else {
                if (g.kind < NK && s >= 0 && s < NS) g.warm_rd[g.kind][s] += 1;
                if (g.lru.size() >= g.lru_cap) {
                    g.lru_pos.erase(g.lru.back());
                    g.lru.pop_back();
                }
            }
            g.lru.push_front(ln);
            g.lru_pos[ln] = g.lru.begin();
        }
    }
    g.in_hook = false;
}
void flush_event() {
    if (g.kind < NK) {
        g.events[g.kind] += 1;
        for (auto& kv : g.rd_sec)
            if (kv.second >= 0 && kv.second < NS) g.cold_rd[g.kind][kv.second] += 1;
        for (auto& kv : g.wr_sec)
            if (kv.second >= 0 && kv.second < NS) g.cold_wr[g.kind][kv.second] += 1;
    }
    g.rd.clear();
    g.wr.clear();
    g.rd_sec.clear();
    g.wr_sec.clear();
}
}  // namespace

extern "C" {
void k10s_tm_replica(const void* base, const void* layout) {
    g.in_hook = true;
    const k10s::Layout& L = *(const k10s::Layout*)layout;
    g.base = (const uint8_t*)base;
    g.stride = L.stride;
    g.hdr_lo = L.hdr;
    g.hdr_hi = L.hdr + sizeof(k10s::RepHdr);
    g.secs.clear();
#define SEC(f) g.secs.push_back({L.f, #f})
    SEC(s_cpu); SEC(s_ram); SEC(s_present); SEC(s_node); SEC(s_bcpu); SEC(s_bram); SEC(s_ccpu); SEC(s_cram);
    SEC(node); SEC(pend_rm); SEC(pod); SEC(prec); SEC(slot); SEC(pool_ring); SEC(grp); SEC(grp_bits);
    SEC(cag); SEC(ca_act); SEC(ca_cpu); SEC(ca_ram); SEC(ca_undo); SEC(ca_ubits); SEC(ca_live); SEC(ps_head);
    SEC(ps_link); SEC(ca_list); SEC(heap); SEC(aq); SEC(uq); SEC(log); SEC(place); SEC(fq); SEC(gauge);
    SEC(g_cpu); SEC(g_ram);
#undef SEC
    std::stable_sort(g.secs.begin(), g.secs.end(), [](const Sec& a, const Sec& b) { return a.off < b.off; });
    g.kind = 0xFFFF;
    g.on = true;
    g.lru.clear();
    g.lru_pos.clear();
    g.in_hook = false;
}
void k10s_tm_event(uint32_t kind) {
    g.in_hook = true;
    flush_event();
    g.kind = kind;
    g.in_hook = false;
}
void k10s_tm_lru(uint32_t lines) { g.lru_cap = lines; }
// JSON: per kind with events, per section cold read lines / cold written 64-B chunks / warm reads.
int k10s_tm_dump(const char* path) {
    g.in_hook = true;
    FILE* f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "{\"sections\": {");
    for (size_t i = 0; i < g.secs.size(); i++)
        fprintf(f, "%s\"%s\": %llu", i ? ", " : "", g.secs[i].name.c_str(), (unsigned long long)g.secs[i].off);
    fprintf(f, "}, \"stride\": %llu, \"kinds\": {", (unsigned long long)g.stride);
    bool first = true;
    for (int k = 0; k < NK; k++) {
        if (g.events[k] == 0) continue;
        fprintf(f, "%s\"%d\": {\"dispatches\": %.0f", first ? "" : ", ", k, g.events[k]);
        first = false;
        const char* nm[4] = {"cold_rd_lines", "cold_wr_chunks", "warm_rd_lines", "raw_loads"};
        double (*tab[4])[NS] = {g.cold_rd, g.cold_wr, g.warm_rd, g.raw_rd};
        for (int t = 0; t < 4; t++) {
            fprintf(f, ", \"%s\": {", nm[t]);
            bool f2 = true;
            for (size_t s = 0; s < g.secs.size() && s < (size_t)NS; s++) {
                if (tab[t][k][s] == 0) continue;
                fprintf(f, "%s\"%s\": %.0f", f2 ? "" : ", ", g.secs[s].name.c_str(), tab[t][k][s]);
                f2 = false;
            }
            fprintf(f, "}");
        }
        fprintf(f, "}");
    }
    fprintf(f, "}}\n");
    fclose(f);
    g.in_hook = false;
    return 0;
}
#define LD(n, T) void __sanitizer_cov_load##n(T* p) { touch(p, false); }
#define STO(n, T) void __sanitizer_cov_store##n(T* p) { touch(p, true); }
LD(1, uint8_t) LD(2, uint16_t) LD(4, uint32_t) LD(8, uint64_t) LD(16, __int128)
STO(1, uint8_t) STO(2, uint16_t) STO(4, uint32_t) STO(8, uint64_t) STO(16, __int128)
void __sanitizer_cov_8bit_counters_init(char*, char*) {}
void __sanitizer_cov_pcs_init(const uintptr_t*, const uintptr_t*) {}
}
