// options.h -- the library's tunables and diagnostic switches, one table per process.
//
// Every value has a compiled-in default, which is what a caller of include/rsync_hip.h gets.  They change only
// through the testing / diagnostics ABI (include/rsync_hip_debug.h: rsh_debug_set_option), never from the
// environment: a stray variable in a user's JVM must not change which kernel or resolver policy runs.  Tests
// use the switches to force paths the default policy takes only on rare shapes (a base next to its
// allocation's start, leftovers one per lane, two launches instead of a segmented one); bench.py --opt and
// the tools use them for same-box A/Bs.  Kernel variants that are not production paths at all are compiled
// only into the kbench tool (RSH_KBENCH), not into librsynchip.so.
#pragma once
#include <stdint.h>
#include <string.h>

#include <atomic>

namespace rsh {

enum Opt : int {
    OPT_K1_GATHER,         // 1: a launch's leftover full-length chunks run as gathered coalesced waves; 0: per lane
    OPT_K1_SHIFT,          // 1: bases off a 128-B line go to the line-aligned shift kernel when it fits the allocation
    OPT_K1_UNALIGNED,      // 1: the pipelined K1 may run at a base that is not 16-B aligned (else per lane)
    OPT_SCAN_TRACE,        // 1: one stderr line per resolver round trip; 2: totals only
    OPT_SCAN_DIAG,         // bit 0: no head mode; bit 1: speculation without an abort word; bit 2: launch at once
    OPT_SCAN_PHASE,        // 1: phase-shifted speculations (chains at kB + delta)
    OPT_SCAN_PHASE_GUESS,  // 1: look for the phase past a sampled run's end before the resolver starts
    OPT_SCAN_SEGMENTED,    // 1: prefix + guessed phase as one segmented K1 launch; 0: two launches
    OPT_SCAN_PREPROBE,     // 1: the probe past the prefix chain rides with the segmented launch
    OPT_SCAN_SAMPLES,      // sampled windows for the speculation launch decision
    OPT_SCAN_SAMPLE,       // 1: cover only the sampled run (prefix speculation)
    OPT_SCAN_SPEC_ORDER,   // 1: the speculation K1 after the sample kernels; 0: beside them
    OPT_SCAN_EARLY,        // 1: launch-then-confirm (the speculation before the host has the table)
    OPT_SCAN_WAIT,         // 1: the resolver waits for a chain-evidence speculation instead of head-mode steps
    OPT_SCAN_DEFER_STEPS,  // head-mode steps before a deferred speculation launch
    OPT_SCAN_DEFER_US,     // ... or this many microseconds
    OPT_BATCH_SPEC,        // batched speculation policy: -1 default, -2 early, -3 wait, N >= 0 launch after N rounds
    OPT_BATCH_SPIN_US,     // round hand-off spin window (0: block at once)
    OPT_BATCH_READAHEAD,   // bytes copied per window request (0: the window only)
    OPT_BATCH_PREP_ALL,    // 1: the batched speculation after all the table work (full-width launches)
    OPT_BATCH_CHAIN,       // 1: the device-side chain advance of the batched scan (batch.cpp)
    OPT_BATCH_CHAIN_PREFIX,  // chain walk over a speculated prefix first (windows per file; -1 auto, 0 off)
    OPT_BATCH_CHAIN_OVERLAP, // 1: the rest of the speculation starts beside the prefix walk (0: after it)
    OPT_HOST_CORES,        // resolver worker threads (0: the process's cores, cgroup quota included)
    OPT_FILE_TILE,         // rsh_match_scan_file: tile bytes above OPT_FILE_TILE_ABOVE
    OPT_FILE_TILE_ABOVE,   // rsh_match_scan_file: sources above this size are scanned tiled
    OPT_PROBE_LONG,        // k > 0: long probe intervals as pass-free segments over ~1024 k workgroups; 0: tiles only
    OPT_SEGMENT_BYTES,     // rsh_*_batch (host memory): bytes of a segment's files copied to HBM per pass
    OPT_MD5_WIDTH,         // rsh_file_md5_batch / rsh_match_scan_batch: 0 = widest multi-buffer MD5, 1/8/16 = forced
    OPT_CHAIN_HELPERS,     // phase-0 walk: extra workgroups mapping searching files' prefixes (-1: CUs - files; 0: no map)
    OPT_CHAIN_MAP_BYTES,   // ... the map's HBM budget (bytes; above it the walks search tile by tile)
    OPT_BATCH_SKIP_REST,   // 1: the rest of a two-phase speculation only if some phase-0 walk reached the prefix's end
    OPT_SCAN_SPEC_QUEUE,   // 1: the single-file speculation on the context stream, round trips on aux; 0: round 4's layout
    OPT_SCAN_FLAGS_HOST,   // 1: (scan_spec_queue) the chain flags kernel writes pinned host memory (no D2H copy)
    OPT_SCAN_PREP_PIECES,  // (scan_spec_queue) workgroups per sampled window in the prep launch (0: auto, <= 8)
    OPT_TIME_SPEC,         // 1: the single-file speculation's K1 records timing events (stats spec_kernel_ms)
    OPT_TIME_GEN,          // 1: rsh_block_sums_device's K1 records timing events (rsh_debug_kernel_ms)
    OPT_FAULT_INJECT,      // tests only: bit 0 a segment / Receiver pass's HBM allocation fails, bit 1 a segment's copies fail
    OPT_COUNT
};

struct OptInfo {
    const char* name;
    int64_t def;
};

inline const OptInfo* opt_info() {
    static const OptInfo t[OPT_COUNT] = {
        {"k1_gather", 1},          {"k1_shift", 1},           {"k1_unaligned", 1},     {"scan_trace", 0},
        {"scan_diag", 0},          {"scan_phase", 1},         {"scan_phase_guess", 1}, {"scan_segmented", 1},
        {"scan_preprobe", 1},      {"scan_samples", 256},     {"scan_sample", 1},      {"scan_spec_order", 1},
        {"scan_early", 1},         {"scan_wait", 1},          {"scan_defer_steps", 4}, {"scan_defer_us", 500},
        {"batch_spec", -1},        {"batch_spin_us", 200},    {"batch_readahead", 0},  {"batch_prep_all", 0},
        {"batch_chain", 1},        {"batch_chain_prefix", -1}, {"batch_chain_overlap", 0},
        {"host_cores", 0},         {"file_tile", 4LL << 30}, {"file_tile_above", 32LL << 30},
        {"probe_long", 1},         {"segment_bytes", 16LL << 30}, {"md5_width", 0},
        {"chain_helpers", -1},     {"chain_map_bytes", 1LL << 30}, {"batch_skip_rest", 1},
        {"scan_spec_queue", 1},    {"scan_flags_host", 1},   {"scan_prep_pieces", 0},   {"time_spec", 0},        {"time_gen", 1},
        {"fault_inject", 0},
    };
    return t;
}

inline std::atomic<int64_t>* opt_table() {
    static std::atomic<int64_t> v[OPT_COUNT] = {};
    static std::atomic<bool> init{false};
    if (!init.load(std::memory_order_acquire)) {
        static std::atomic_flag once = ATOMIC_FLAG_INIT;
        if (!once.test_and_set()) {
            for (int i = 0; i < OPT_COUNT; ++i) v[i].store(opt_info()[i].def, std::memory_order_relaxed);
            init.store(true, std::memory_order_release);
        } else {
            while (!init.load(std::memory_order_acquire)) {
            }
        }
    }
    return v;
}

inline int64_t opt(Opt o) { return opt_table()[o].load(std::memory_order_relaxed); }

// -1 when the name is unknown
inline int opt_index(const char* name) {
    for (int i = 0; i < OPT_COUNT; ++i)
        if (name && strcmp(name, opt_info()[i].name) == 0) return i;
    return -1;
}

}  // namespace rsh
