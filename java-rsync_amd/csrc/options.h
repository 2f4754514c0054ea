// options.h -- the library's tunables and diagnostic switches, one table per process.
//
// Every value has a compiled-in default, which is what a caller of include/rsync_hip.h gets.  They change only
// through the testing / diagnostics ABI (include/rsync_hip_debug.h: rsh_debug_set_option), never from the
// environment: a stray variable in a user's JVM must not change which kernel or resolver policy runs.
//
// Two kinds:
//  * switches the product library reads at run time: tests set them to force paths the default policy takes only
//    on rare shapes (a base next to its allocation's start, leftovers one per lane, two launches instead of a
//    segmented one, a file larger than a pass) or to inject a failure; a few are tunables (budgets, cores);
//  * A/B switches (ab = true): the alternatives a measurement rejected and the policies' knobs, kept for same-box
//    A/Bs.  The product build reads their compiled-in default as a constant (the branches they guard are dead
//    code, and rsh_debug_set_option refuses them); the diagnostics build (make diag: -DRSH_DIAG,
//    lib/diag/librsynchip.so, which the tools load through RSH_LIB) reads them from the table.
// Kernel variants that are not production paths at all are compiled only into the kbench tool (RSH_KBENCH).
#pragma once
#include <stdint.h>
#include <string.h>

#include <atomic>

namespace rsh {

enum Opt : int {
    // ---- read by the product library ----
    OPT_K1_GATHER,         // 1: a launch's leftover full-length chunks run as gathered coalesced waves; 0: per lane
    OPT_K1_SHIFT,          // 1: bases off a 128-B line go to the line-aligned shift kernel when it fits the allocation
    OPT_K1_UNALIGNED,      // 1: the pipelined K1 may run at a base that is not 16-B aligned (else per lane)
    OPT_SCAN_TRACE,        // 1: one stderr line per resolver round trip; 2: totals only
    OPT_SCAN_SEGMENTED,    // 1: prefix + guessed phase as one segmented K1 launch; 0: two launches
    OPT_SCAN_SAMPLES,      // sampled windows for the speculation launch decision
    OPT_BATCH_CHAIN,       // 1: the device-side chain advance of the batched scan (batch.cpp)
    OPT_BATCH_CHAIN_PREFIX,  // chain walk over a speculated prefix first (windows per file; -1 auto, 0 off)
    OPT_HOST_CORES,        // resolver worker threads (0: the process's cores, cgroup quota included)
    OPT_FILE_TILE,         // rsh_match_scan_file: tile bytes above OPT_FILE_TILE_ABOVE
    OPT_FILE_TILE_ABOVE,   // rsh_match_scan_file: sources above this size are scanned tiled
    OPT_PROBE_LONG,        // k > 0: long probe intervals as pass-free segments over ~1024 k workgroups; 0: tiles only
    OPT_SEGMENT_BYTES,     // rsh_*_batch (host memory): bytes of a segment's files copied to HBM per pass
    OPT_MD5_WIDTH,         // rsh_file_md5_batch / rsh_match_scan_batch: 0 = widest multi-buffer MD5, 1/8/16 = forced
    OPT_CHAIN_HELPERS,     // phase-0 walk: extra workgroups mapping searching files' prefixes (-1: CUs - files; 0: no map)
    OPT_CHAIN_MAP_BYTES,   // ... the map's HBM budget (bytes; above it the walks search tile by tile)
    OPT_TIME_GEN,          // 1: rsh_block_sums_device's K1 records timing events (rsh_debug_kernel_ms)
    OPT_BATCH_WARM,        // rsh_ctx_create pre-sizes the batched scan's state for this many 128 MiB files (0: none)
    OPT_FAULT_INJECT,      // tests only: bit 0 a segment / Receiver pass's HBM allocation fails, bit 1 a segment's copies fail,
                           // bit 2 bits 0 / 1 only on member 1 of a multi-context call (multi.cpp)
    // ---- A/B switches (the diagnostics build reads them; the product build uses the defaults) ----
    OPT_SCAN_DIAG,         // bit 0: no head mode; bit 1: speculation without an abort word; bit 2: launch at once
    OPT_SCAN_PHASE,        // 1: phase-shifted speculations (chains at kB + delta)
    OPT_SCAN_PHASE_GUESS,  // 1: look for the phase past a sampled run's end before the resolver starts
    OPT_SCAN_PREPROBE,     // 1: the probe past the prefix chain rides with the segmented launch
    OPT_SCAN_SAMPLE,       // 1: cover only the sampled run (prefix speculation)
    OPT_SCAN_SPEC_ORDER,   // (scan_spec_queue 0) 1: the speculation K1 after the sample kernels; 0: beside them
    OPT_SCAN_EARLY,        // 1: launch-then-confirm (the speculation before the host has the table)
    OPT_SCAN_WAIT,         // 1: the resolver waits for a chain-evidence speculation instead of head-mode steps
    OPT_SCAN_DEFER_STEPS,  // head-mode steps before a deferred speculation launch
    OPT_SCAN_DEFER_US,     // ... or this many microseconds
    OPT_SCAN_SPEC_QUEUE,   // 1: the single-file speculation on the context stream, round trips on aux; 0: round 4's layout
    OPT_SCAN_FLAGS_HOST,   // 1: (scan_spec_queue) the chain flags kernel writes pinned host memory (no D2H copy)
    OPT_SCAN_PREP_PIECES,  // (scan_spec_queue) workgroups per sampled window in the prep launch (0: auto, <= 8)
    OPT_TIME_SPEC,         // 1: the single-file speculation's K1 records timing events (stats spec_kernel_ms)
    OPT_BATCH_SPEC,        // batched speculation policy: -1 default, -2 early, -3 wait, N >= 0 launch after N rounds
    OPT_BATCH_SPIN_US,     // round hand-off spin window (0: block at once)
    OPT_BATCH_READAHEAD,   // bytes copied per window request (0: the window only)
    OPT_BATCH_PREP_ALL,    // 1: the batched speculation after all the table work (full-width launches)
    OPT_BATCH_CHAIN_OVERLAP, // 1: the rest of the speculation starts beside the prefix walk (0: after it)
    OPT_BATCH_SKIP_REST,   // 1: the rest of a two-phase speculation only if some phase-0 walk reached the prefix's end
    OPT_CHAIN_HELP_TILES,  // tiles a phase-0 walk searches before helpers map ahead of it
    OPT_COUNT
};

struct OptInfo {
    const char* name;
    int64_t def;
    bool ab;  // an A/B switch: settable in the diagnostics build only
};

inline constexpr OptInfo kOpts[OPT_COUNT] = {
    {"k1_gather", 1, false},          {"k1_shift", 1, false},        {"k1_unaligned", 1, false},
    {"scan_trace", 0, false},         {"scan_segmented", 1, false},  {"scan_samples", 256, false},
    {"batch_chain", 1, false},        {"batch_chain_prefix", -1, false}, {"host_cores", 0, false},
    {"file_tile", 4LL << 30, false},  {"file_tile_above", 32LL << 30, false}, {"probe_long", 1, false},
    {"segment_bytes", 16LL << 30, false}, {"md5_width", 0, false}, {"chain_helpers", -1, false},
    {"chain_map_bytes", 1LL << 30, false}, {"time_gen", 1, false}, {"batch_warm", 128, false},
    {"fault_inject", 0, false},
    {"scan_diag", 0, true},           {"scan_phase", 1, true},       {"scan_phase_guess", 1, true},
    {"scan_preprobe", 1, true},       {"scan_sample", 1, true},      {"scan_spec_order", 1, true},
    {"scan_early", 1, true},          {"scan_wait", 1, true},        {"scan_defer_steps", 4, true},
    {"scan_defer_us", 500, true},     {"scan_spec_queue", 1, true},  {"scan_flags_host", 1, true},
    {"scan_prep_pieces", 0, true},    {"time_spec", 0, true},        {"batch_spec", -1, true},
    {"batch_spin_us", 200, true},     {"batch_readahead", 0, true},  {"batch_prep_all", 0, true},
    {"batch_chain_overlap", 0, true}, {"batch_skip_rest", 1, true},  {"chain_help_tiles", 1, true},
};

#ifdef RSH_DIAG
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif

inline const OptInfo* opt_info() { return kOpts; }

inline std::atomic<int64_t>* opt_table() {
    static std::atomic<int64_t> v[OPT_COUNT] = {};
    static std::atomic<bool> init{false};
    if (!init.load(std::memory_order_acquire)) {
        static std::atomic_flag once = ATOMIC_FLAG_INIT;
        if (!once.test_and_set()) {
            for (int i = 0; i < OPT_COUNT; ++i) v[i].store(kOpts[i].def, std::memory_order_relaxed);
            init.store(true, std::memory_order_release);
        } else {
            while (!init.load(std::memory_order_acquire)) {
            }
        }
    }
    return v;
}

// An A/B switch in the product build is its compiled-in default (a constant: the branches it guards fold away).
inline int64_t opt(Opt o) {
    if (!kDiagBuild && kOpts[o].ab) return kOpts[o].def;
    return opt_table()[o].load(std::memory_order_relaxed);
}

// -1 when the name is unknown
inline int opt_index(const char* name) {
    for (int i = 0; i < OPT_COUNT; ++i)
        if (name && strcmp(name, kOpts[i].name) == 0) return i;
    return -1;
}

// rsh_debug_set_option may change it in this build
inline bool opt_settable(int i) { return i >= 0 && i < OPT_COUNT && (kDiagBuild || !kOpts[i].ab); }

}  // namespace rsh
