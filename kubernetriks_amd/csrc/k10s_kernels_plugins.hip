// k10s_kernels_plugins.hip — the event-loop kernels (init + run) compiled a second time with the
// score-plugin profile path in (K10S_SCORE_PLUGINS=1: MostAllocatedResources and multi-plugin
// profiles, k10s_engine.h run_scheduling_cycle_plugins) and the wide node-cache layout
// (K10S_PACKED=0).  Symbols are renamed so both copies live in one library; k10s_host.cpp launches
// this copy for engines with such a replica or whose node cache is not packed (Layout.packed).  Every engine
// function and type of this copy lives in namespace k10s_plugins (the `k10s` token renamed), so the
// two copies' handlers — different bodies of the same inline functions — never share a mangled
// name (no ODR clash if the library is ever linked with -fgpu-rdc or LTO).
#define k10s k10s_plugins
#define K10S_SCORE_PLUGINS 1
#define K10S_PACKED 0   // the wide node cache (u32 cpu + u64 ram SoA): plugin replicas read the capacity
                        // SoA beside it, and scenarios whose nodes do not fit the packed entry run here
#define K10S_PLUGINS_TU 1
#define K10S_TIME_KEY_ID 0   // the general total_cmp key: scenarios with signed event times run here
#define k10s_dc k10s_dc_plugins
#define k10s_hdr k10s_hdr_plugins
#define k10s_sec k10s_sec_plugins
#define k10s_fair_board k10s_fair_board_plugins
#define k10s_beacon k10s_beacon_plugins   // (K10S_BEACON tooling builds) this copy's own pointer, set with the other
#define k10s_run k10s_run_plugins
#define k10s_init_kernel k10s_init_kernel_plugins
#define k10s_run_kernel k10s_run_kernel_plugins
#define k10s_launch_init k10s_launch_init_plugins
#define k10s_launch_run k10s_launch_run_plugins
#include "k10s_kernels.hip"
