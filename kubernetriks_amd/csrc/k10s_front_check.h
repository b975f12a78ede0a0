// The invariant of the per-block Pareto fronts (k10s_engine.h fr_block / fr_refresh), recomputed from
// a replica's node cache: test support for k10s_engine_check_fronts (device state) and the test-only
// host engine (tests/hostcheck), not part of the event loop.
#pragma once
#include <cstdint>

// Every block not marked stale in `dirty` must hold exactly its index-aware front in its K slots
// (a node is in the front iff no later node of its block has at least as much free cpu and free
// ram; the first K front nodes in node order, unused slots 0) and its `over` bit must say whether the
// front is longer than K.  Returns the number of blocks checked, or -(1 + the first block that
// breaks it).  sn: the packed entries (cpu << 40 | ram); fv / fi: the slots and their offsets.
inline int32_t k10s_front_check(const uint64_t* sn, const uint64_t* fv, const uint8_t* fi, uint32_t N, uint64_t dirty,
                                uint64_t over, uint32_t K) {
    const uint64_t ram_mask = (1ull << 40) - 1;
    int32_t checked = 0;
    for (uint32_t b = 0; 64u * b < N && b < 64u; b++) {
        if ((dirty >> b) & 1ull) continue;
        const uint32_t lo = 64u * b, hi = lo + 64u < N ? lo + 64u : N;
        uint32_t mem[64];
        uint32_t nf = 0;
        for (uint32_t k = hi; k-- > lo;) {   // from the last node: kept iff no kept later node dominates it
            const uint64_t x = sn[k];
            if (x == 0) continue;
            bool dom = false;
            for (uint32_t q = 0; q < nf && !dom; q++) {
                const uint64_t w = sn[mem[q]];
                dom = (w >> 40) >= (x >> 40) && (w & ram_mask) >= (x & ram_mask);
            }
            if (!dom) mem[nf++] = k;
        }
        bool ok = ((over >> b) & 1ull) == (nf > K ? 1ull : 0ull);
        for (uint32_t s = 0; s < K && ok; s++) {
            if (s < nf) {
                const uint32_t k = mem[nf - 1 - s];
                ok = fv[b * K + s] == sn[k] && fi[b * K + s] == (uint8_t)(k - lo);
            } else {
                ok = fv[b * K + s] == 0;
            }
        }
        if (!ok) return -(1 + (int32_t)b);
        checked++;
    }
    return checked;
}
