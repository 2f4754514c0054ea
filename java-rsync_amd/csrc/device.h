// device.h -- internal launchers for the gfx950 kernels in device.hip (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "hit_cache.h"
#include "rsync_hip.h"

namespace rsh {

// Generator block sums (Generator.java:886-895): chunk c covers [c*B, min((c+1)*B, n)).
// Writes weak[c] and strong[c*dl .. c*dl+dl).  Also used by the Sender as aligned speculation.
// abort_flag (optional, host-pinned): the launch stops early, leaving its outputs undefined, once
// *abort_flag == abort_gen (the Sender's speculation when the resolver no longer needs it).
hipError_t launch_block_sums(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks, uint32_t dl,
                             uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong, hipStream_t s,
                             const int* abort_flag = nullptr, int abort_gen = 0);
// Timing of the next K1 launch_block_sums makes on this thread: its dispatch records start / stop in these events
// (hipExtLaunchKernelGGL: the kernel's own timestamps, no marker packets in the stream and so no bubble before or
// after the kernel).  k1_timing_taken() says whether that launch took them (the pipelined and the shift kernels do;
// the rare per-lane and coalesced shapes do not, and the events then stay unrecorded).
void k1_timing_next(hipEvent_t start, hipEvent_t stop);
bool k1_timing_taken();

#ifdef RSH_KBENCH
// kbench only (tools/kbench.cpp, built with -DRSH_KBENCH): the single-file K1 launcher with its variant exposed
// (-1 = production, 0 = every chunk per lane, kbench's parity reference).
hipError_t launch_block_sums_variant(int variant, const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks,
                                     uint32_t dl, uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong,
                                     hipStream_t s, const int* abort_flag = nullptr, int abort_gen = 0);
#endif

// Batched files (a segment's files in one launch; Generator.java:558-614 / Sender.sendFiles :1098-1148).
// K1File: one file's chunk set.  plan_block_sums_batch cuts every file into waves of 64 chunks: the
// pipelined coalesced K1 (K1Group: 64 full-length chunks, B % 128 == 0, 512 <= B <= 128 KiB, 16-B aligned
// data) and one lane per chunk for the rest (K1Lane: the file's tail group, or every chunk of a file
// whose shape the coalesced kernel does not take).  The descriptors must be device-readable.
struct K1File {
    const uint8_t* data;
    int64_t n;
    uint32_t B, dl, nchunks;
    int32_t* weak;
    uint8_t* strong;
};
struct K1Group {
    const uint8_t* data;  // chunk 0 of the group
    int32_t* weak;        // its output slots
    uint8_t* strong;
    uint32_t B, dl;
    const int* abort = nullptr;  // abortable launches: this group's own abort word (nullptr: the launch's)
    int32_t file = 0;            // index of its file in the planner's list (host bookkeeping only)
    uint32_t count = 64;         // its chunks (< 64: a file's partial last wave, run as a gathered wave)
};
struct K1Lane {
    const uint8_t* data;  // the file
    int64_t n;
    int32_t* weak;        // the file's output arrays
    uint8_t* strong;
    uint32_t B, dl, c_first, nchunks;
    int32_t file = 0;     // index of its file in the planner's list (host bookkeeping only)
};
// Segmented K1 (the Sender's prefix + phase-shifted speculation in one launch): K1Seg = one wave of 64 full
// chunks of length B starting at lines + a (lines 128-B aligned, [lines, lines + 64 B + 128) readable), with
// its own output slots and abort word; K1Tail = one leftover chunk (chunk c of the file (data, n)).
struct K1Seg {
    const uint8_t* lines;
    int32_t* weak;
    uint8_t* strong;
    const int* abort;
    int32_t abort_gen;
    uint32_t a;
};
struct K1Tail {
    const uint8_t* data;
    int64_t n;
    int32_t* weak;  // the file's output arrays (chunk c is written at weak[c], strong[c * dl])
    uint8_t* strong;
    uint32_t c;
};
// d_tails[0, nfull): full-length chunks (gathered 64 to a coalesced wave when that adds no wave); the rest
// (short chunks) one per lane
hipError_t launch_block_sums_segments(const K1Seg* d_segs, uint32_t nseg, const K1Tail* d_tails, uint32_t ntail,
                                      uint32_t nfull, uint32_t B, uint32_t dl, uint32_t seed_word, hipStream_t s);
void plan_block_sums_batch(const K1File* files, int32_t nfiles, std::vector<K1Group>* groups,
                           std::vector<K1Lane>* lanes, int* lane_align);
// Device-side group expansion: the host plans per file (K1Plan: the file's first group index g0 and its
// count of full 64-chunk groups) and one thread per group writes its K1Group (expand_groups_kernel), instead of
// the host building and uploading ~40 B per 64 chunks (config 4: 32768 groups, 1.5 MB, ~0.14 ms of host time
// per batched call).  Lanes (tails, odd shapes) stay host-planned: they are few.
struct K1Plan {
    const uint8_t* data;
    int32_t* weak;
    uint8_t* strong;
    uint32_t B, dl;
    uint32_t g0, ng;            // groups [g0, g0 + ng) of the launch are this file's chunks [0, min(64 ng, nfull))
    const int* abort = nullptr;  // K1Group::abort of its groups
    int32_t file = 0;
    uint32_t nfull = 0;          // its full-length chunks covered by groups (the last group may be partial)
};
// plans (one per file with groups, ascending g0) and the host lanes; returns the total group count.  A file's
// full-length chunks past its last full wave form a partial group (K1Group::count < 64) when *partial is set
// on entry (option k1_gather); on return *partial says whether any plan has one.
uint32_t plan_block_sums_files(const K1File* files, int32_t nfiles, std::vector<K1Plan>* plans,
                               std::vector<K1Lane>* lanes, int* lane_align, bool* partial = nullptr);
hipError_t launch_expand_groups(const K1Plan* d_plans, uint32_t nplans, uint32_t ngroups, K1Group* d_groups,
                                hipStream_t s);
bool tail_gather_on();  // option k1_gather = 0: leftover chunks one per lane, no gathered waves
// partial: some groups have count < 64 (plan_block_sums_files) -- they run as gathered waves of the same launch
hipError_t launch_block_sums_batch(const K1Group* d_groups, uint32_t ngroups, const K1Lane* d_lanes, uint32_t nlanes,
                                   int lane_align, uint32_t seed_word, hipStream_t s, const int* abort_flag = nullptr,
                                   int abort_gen = 0, bool partial = false);

// Chain flags for the Sender fast path: flag[k] = 1 iff source window k (aligned, from the source's
// own block sums) has the same weak key and the same dl-byte digest as basis chunk k.
hipError_t launch_chain_flags(const int32_t* d_wsrc, const uint8_t* d_ssrc, const int32_t* d_wbas,
                              const uint8_t* d_sbas, uint32_t count, uint32_t dl, uint8_t* d_flags,
                              hipStream_t s);
// One empty kernel per code object (device.hip, device_scan.hip, device_io.hip): rsh_ctx_create launches them so that
// the runtime loads every production kernel before the first call.
hipError_t launch_warm_k1(hipStream_t s);
hipError_t launch_warm_scan(hipStream_t s);
hipError_t launch_warm_chain(hipStream_t s);
hipError_t launch_warm_io(hipStream_t s);
// Completion without a marker packet: the launch's last workgroup to finish writes `gen` into *stamp (pinned host
// memory, system-scope release after every workgroup's stores), which the host polls.  counter: device memory,
// zero before the launch (the last workgroup zeroes it again).
// counter: kStampLine * (1 + kStampGroups) device words, zero between launches (the launch counter, then the group
// counters of device_io.hip stamp_arrive, a 64-B line each)
constexpr uint32_t kStampGroups = 64, kStampLine = 16;
struct Stamp {
    uint32_t* counter;
    int* stamp;
    int gen;
};
// The chain flags of the single-file scan into pinned host memory, stamped.
hipError_t launch_chain_flags_stamped(const int32_t* d_wsrc, const uint8_t* d_ssrc, const int32_t* d_wbas,
                                      const uint8_t* d_sbas, uint32_t count, uint32_t dl, uint8_t* h_flags,
                                      Stamp st, hipStream_t s);
// The single-file scan's launch decision in one launch on the speculation's queue, ahead of it (scan_device,
// scan_spec_queue): the weak sums T(kB) of the sampled windows wins[i] (each window split over `pieces` workgroups,
// partial sums added with device atomics into scratch, 2 ints per sample, zero before the launch), the received
// table's weak sums at the same chunks, and window 0's bytes, all into pinned host memory, then the stamp.
struct ScanPrep {
    const uint8_t* data;
    int64_t n;
    uint32_t B;
    uint32_t nsamp, pieces;
    // the sampled windows: i < nlead: window i; then window stride * (j0 + i - nlead) (capi.cpp scan_device's list)
    uint32_t nlead;
    int64_t stride, j0;
    const int32_t* table_weak;  // device: the received table's weak sums
    int32_t C;
    int32_t* out_t;             // pinned host: T(wins[i] B)
    int32_t* out_w;             // pinned host: table_weak[wins[i]] (0 past the table)
    uint8_t* w0;                // pinned host: window 0 (w0_len bytes)
    int64_t w0_len;
    int32_t* scratch;           // device: 2 nsamp ints
    Stamp st;
};
hipError_t launch_scan_prep(const ScanPrep& P, hipStream_t s);

// Probe table: open-addressing hash of the distinct weak keys (key -> 1).  slots = power of two.
struct ProbeTable {
    const unsigned long long* slots;
    uint32_t mask;
};
// bg (background): priority 0 and at most kBackgroundGroups workgroups, for table work that runs beside a K1
// launch (a high-priority kernel spread over every CU slows the K1 waves that share its SIMDs, and the slowest
// wave ends the launch)
constexpr uint32_t kBackgroundGroups = 256;
hipError_t launch_table_clear(unsigned long long* d_slots, uint64_t nslots, hipStream_t s, bool bg = false);
hipError_t launch_table_insert(unsigned long long* d_slots, uint32_t mask, const int32_t* d_keys, uint32_t nkeys,
                               hipStream_t s);

// Sender-side rolling key probe.  For each interval [a, b) the key is R(p) = T(p) + E(p), where T(p) is
// the true weak sum of window [p, p + min(B, n - p)) and E(p) = (e_lo, e_hi + e_lo * (min(p, n-B) -
// min(anchor, n-B))) mod 2^16 (the post-flush desync of Sender.java:1292-1310).  The work is cut into
// tiles of PROBE_TILE positions inside aligned blocks [kB, kB + B); aligned_weak[k] = T(kB) (the
// source's own block sums) anchors each block.  The file's ProbeOut receives the smallest hitting position
// over all its tiles and the list of hits.
//
// One launch serves a batch of files (a round of the batched Sender, or a single scan as a batch of one):
// every interval names its file, and a file's per-scan state is a ScanFile in device-readable memory.
constexpr int PROBE_TILE = 4096;
// Tiles at most this far into their block take their block prefix by re-reading the tiles before them
// (<= 2 x PROBE_INLINE_TILES x 4 KiB) instead of from pass 1; blocks of B <= 8 KiB then need no pass 1.
constexpr int PROBE_INLINE_TILES = 1;
constexpr int HIT_BUCKET_CAP = 256;
constexpr int HIT_BUCKET_INTS = 2 + HIT_BUCKET_CAP + PROBE_HITS_CAP * (1 + LISTED_IDX);
constexpr int PROBE_SMALL_KEYS = 8;
struct ScanFile {
    const uint8_t* data;
    int64_t n;
    uint32_t B;
    uint32_t mask;                    // the round's probe key set: slots[0 .. mask]
    const unsigned long long* slots;
    int32_t* aligned_weak;            // T(kB) anchors (the speculation's weak sums, or head-mode window sums)
    ProbeOut* out;                    // probe result (device)
    const int32_t* table_weak;        // the received table's weak sums (device), C entries
    int32_t C;
    int32_t iv0, niv;                 // the file's intervals in the round's ProbeIv array
    int32_t nwin;                     // hit windows wanted (1 .. HIT_WINDOWS)
    int32_t* bucket;                  // device, HIT_BUCKET_INTS: {count, key, idx[0 .. HIT_BUCKET_CAP)} of the
                                      // first hit, then per listed hit j {count, idx[LISTED_IDX]}
    uint8_t* hit;                     // pinned host: T(p) in bytes 0..3, window k of the k-th smallest listed
                                      // hit at 16 + k B (k < HIT_WINDOWS; k = 0: the first hit)
    int32_t next_sums;                // 0..NEXT_SUMS_MAX: T(p + k B) of the first hit p for k = 1..next_sums too, into hit bytes 4 k
                                      // (the phase guess's check of four consecutive windows in the same round trip)
    int32_t nsmall;                   // > 0: the round's key set is these few keys (a stale digest's chunks),
    uint32_t small[PROBE_SMALL_KEYS]; // compared in registers instead of looked up in slots
};
struct ProbeIv {
    int64_t a, b, anchor;
    uint32_t e_lo, e_hi;
    int32_t file;
    int32_t pad;
};
// The batched flush chain on the device (device_scan.hip flush_chain_kernel; resolver.h FlushChain): from the
// gathered T(f_i), T(f_i + B) and the bytes at f_i, f_i + 2B - 1, every step's desync (elo, ehi) into out[2i, 2i+1]
// and into the e_lo / e_hi of the chain's probe intervals iv[0, niv) -- in stream order before the probe reads them.
struct FlushChainJob {
    const int32_t* tv;  // 2K weak sums (device memory)
    const uint8_t* bv;  // 2K bytes (device memory)
    ProbeIv* iv;        // where the probe reads the chain's intervals
    uint32_t* out;      // 2K words (pinned host memory: the resolver commits the flushes from them)
    int64_t f, B, n, last;
    int32_t K, niv;
    uint32_t el, eh;
};
hipError_t launch_flush_chain(const FlushChainJob* jobs, uint32_t njobs, hipStream_t s);
struct ProbeTile {
    int64_t q0;     // tile start (multiple of PROBE_TILE from its block start)
    int32_t iv;     // interval index
    int32_t pbase;  // index of its block's tile-0 partial sums in ProbeArgs::partials; -1: computed in-kernel
};
// Pass 1 of a probe: the four byte sums (x[j], (j - o) x[j] over the tile, and the same over the tile
// shifted by B) of every tile of a block that lies before a probed tile of that block, so that pass 2
// gets each tile's block prefix from at most 31 partials instead of re-reading up to B bytes per tile.
struct PartialTile {
    int64_t q0;
    int32_t file;
    int32_t pad;
};
struct ProbeArgs {
    const ScanFile* files;
    const ProbeIv* ivs;
    const ProbeTile* tiles;
    int4* partials;  // written by pass 1
};
// Long intervals (a batched flush chain over a file's rest: ~1600 intervals of 9B + 1 positions) as segments of up
// to PROBE_LONG_PASSES x PROBE_LONG_SUB positions, one workgroup each, PROBE_LONG_PPL consecutive positions per lane: the workgroup
// digests its own anchor T(q0) (the window at its first position) instead of taking it from an aligned block's
// sums, so segments ignore block boundaries and need no pass 1.  Only positions whose window is full (p <= n - B).
constexpr int PROBE_LONG_PPL = 64;
constexpr int64_t PROBE_LONG_SUB = 256 * PROBE_LONG_PPL;  // positions per pass of a workgroup's lanes
constexpr int64_t PROBE_LONG_PASSES = 8;                  // at most this many passes per workgroup (one anchor)
constexpr int64_t PROBE_LONG_MIN = 2 * PROBE_LONG_SUB;    // shorter full-window parts stay in tiles
constexpr int64_t PROBE_LONG_BIG = 256 * PROBE_LONG_SUB;  // smaller probes stay in tiles (parallelism, latency)
constexpr int64_t PROBE_LONG_MAX_B = 16384;               // larger blocks stay in tiles (the anchor reads B bytes)
struct ProbeSeg {
    int64_t q0;   // first position (16-aligned; positions below the interval's a are skipped)
    int32_t iv;   // interval index
    int32_t len;  // positions [q0, q0 + len), every one <= n - B
};
// Appends the tiles covering [a, b) for interval `iv` (host side).
void probe_tiles(int64_t a, int64_t b, int64_t B, int32_t iv, std::vector<ProbeTile>* out);
// The segment length for a probe whose intervals hold `full_positions` full-window positions in all (0: tiles only).
int64_t probe_seg_len(int64_t full_positions, int64_t B);
int64_t probe_full_positions(int64_t a, int64_t b, int64_t n, int64_t B);
// As probe_tiles, with the full-window part of a long interval as segments of seg_len positions (host side).
void probe_plan(int64_t a, int64_t b, int64_t n, int64_t B, int32_t iv, int64_t seg_len, std::vector<ProbeTile>* tiles,
                std::vector<ProbeSeg>* segs);
// The segments' launch (writes the same ProbeOut records as the tiles' launch; either order).
hipError_t launch_probe_long(const ProbeArgs& args, const ProbeSeg* segs, uint32_t nsegs, hipStream_t s);
// Assigns ProbeTile::pbase for tiles[t0 ..] (one file's tiles, ascending) and appends the partial tiles
// pass 1 computes for them (host side).
void probe_partials(std::vector<ProbeTile>* tiles, size_t t0, int64_t B, int32_t file, std::vector<PartialTile>* out);
// Both passes, back to back on stream s.
hipError_t launch_probe_first(const ProbeArgs& args, uint32_t ntiles, const PartialTile* ptiles, uint32_t nptiles,
                              hipStream_t s);
// After a probe, for each file req[r] (r < nreq) whose *first holds a position p: the resolver's next
// questions answered in the same round trip: the true weak sum T(p) and the window [p, p + min(B, n - p))
// into the file's pinned `hit` buffer, and the bucket of the key R(p) = T(p) + E(p) (E from the interval
// holding p) in the received table: bucket = {count, key, idx[0 .. min(count, cap))}, in no particular
// order.  max_C: the largest C among the files.
hipError_t launch_hit_window(const ScanFile* files, const ProbeIv* ivs, const int32_t* req, int32_t nreq, int32_t max_C,
                             hipStream_t s);

// Presets n ProbeOut records (first = ~0, count = 0).
hipError_t launch_probe_out_reset(ProbeOut* d_out, uint32_t n, hipStream_t s);

// Small gathers for a batch of files (pinned-host or device entries; outputs in device-readable memory).
struct GatherEnt {
    int64_t p;
    int32_t file;
    int32_t by_block;  // window_weak: 1 = write files[file].aligned_weak[p / B] instead of out[i]
};
// Bytes at arbitrary positions: out[i] = files[e.file].data[e.p].
hipError_t launch_gather_bytes(const ScanFile* files, const GatherEnt* ents, uint32_t n, uint8_t* out, hipStream_t s);
// True weak sums at arbitrary positions: Rolling.compute(data + p, min(B, n - p)).
hipError_t launch_window_weak(const ScanFile* files, const GatherEnt* ents, uint32_t n, int32_t* out, hipStream_t s);
// Many device ranges into pinned host memory (or device memory), one kernel.
struct CopyEnt {
    const uint8_t* src;
    uint8_t* dst;
    int64_t len;
};
hipError_t launch_copy_many(const CopyEnt* ents, uint32_t n, int64_t max_len, hipStream_t s, bool bg = false);
// Up to four device ranges into pinned host memory, the ranges passed by value in the kernel's arguments (nothing
// for the host to keep alive after the launch); any alignment of source and destination.
struct CopyFew {
    CopyEnt e[4];
    uint32_t n;
};
hipError_t launch_copy_few(const CopyFew& f, hipStream_t s);
// The same ranges by one workgroup, then `gen` into the pinned `stamp` (the host spins on it).
hipError_t launch_copy_few_stamped(const CopyFew& f, int* stamp, int gen, hipStream_t s);
// n bytes of device memory into pinned host memory (h_dst 16-byte aligned), by a kernel.
hipError_t launch_copy_to_host(const uint8_t* d_src, int64_t n, uint8_t* h_dst, hipStream_t s);
// Byte ranges between arbitrary (unaligned) device addresses: one op per workgroup, 16-byte stores to
// the aligned middle of each destination (Receiver block gather).
struct GatherOp {
    const uint8_t* src;
    uint8_t* dst;
    int64_t len;
};
// avg_len (optional): the ops' average length; below 64 KiB a 256-thread form (four short ops per CU slot of one)
hipError_t launch_gather_ops(const GatherOp* ops, uint32_t n, hipStream_t s, int64_t avg_len = 1 << 20);
#ifdef RSH_KBENCH
hipError_t launch_gather_ops_variant(int v, const GatherOp* ops, uint32_t n, hipStream_t s);  // A/Bs (kbench)
#endif
// Probe hashes of many files (slots cleared by the caller): keys[i] into slots/mask.
struct TableEnt {
    unsigned long long* slots;
    const int32_t* keys;
    uint32_t mask;
    int32_t nkeys;
};
hipError_t launch_table_insert_many(const TableEnt* ents, uint32_t n, int32_t max_keys, hipStream_t s,
                                    bool bg = false);
// Chain flags of many files.
struct FlagEnt {
    const int32_t* wsrc;
    const uint8_t* ssrc;
    const int32_t* wbas;
    const uint8_t* sbas;
    uint8_t* flags;
    uint32_t count, dl;
};
hipError_t launch_chain_flags_many(const FlagEnt* ents, uint32_t n, uint32_t max_count, hipStream_t s);
// Host mirror of the device probe hash (key sets built on the host, e.g. the stale-digest keys).
inline uint32_t slot_hash_host(uint32_t key) {
    const uint32_t h = key * 0x9E3779B1u;
    return h ^ (h >> 15);
}

// Chain advance of a batched Sender scan (device.hip chain_advance_kernel, batch.cpp): one workgroup per file
// walks Sender.sendMatchesAndData on the device while the state stays synced and unpoisoned and every digest
// comes from the aligned speculation; it stops before any other step, which the host resolver then takes.
// ChainOut holds the state on entry (s, m, pref) and on return; events go to ev (device-readable, ev_cap).
// CHAIN_MORE: the walk reached the end of a prefix speculation (phase 0); phase 1 resumes it over the whole file
enum { CHAIN_STOP = 0, CHAIN_DONE = 1, CHAIN_MORE = 2 };
constexpr int CHAIN_BUCKET_CAP = 64;
struct ChainOut {
    int64_t s, m;
    int32_t pref, status;
    int32_t n_ev, tiles;  // tiles: probe tiles the walk searched (trace)
    int64_t literal, matched, chain_matches, events;
    // stopped on a poisoned state (quirk B): the stale cached digest, the window's at the hit (md5c_valid = 1)
    uint8_t md5c[16];
    int32_t md5c_valid, digests;  // digests: windows the walk digested itself (unaligned hits)
    int64_t flushes;              // FileView flushes of the closed form (a dead poisoned state)
    int64_t t_total, t_tiles, t_check, t_event, t_digest;  // wall-clock ticks (10 ns) of the walk's parts (trace)
    int64_t t_kset, t_chain, t_drain;  // ... the key set's build, steps (1) and (1'), the event drains (trace)
    int64_t t_evb;                     // ... the events' first part: their bucket's load and barrier (trace)
    int32_t spec_full;            // phase 1 walked it
    int32_t aborted;              // phase 0 stopped its phase-1 K1 groups: only the prefix is speculated
    int32_t mapped, first_mapped; // tiles answered from the hit map; the walk's tile count at the first (trace)
    int64_t clear_to;             // stopped before a flush: no candidate in [s, clear_to] (else -1)
    int32_t why, pad2;            // why the walk stopped (CHAIN_WHY_*, trace)
    uint32_t elo, ehi;            // CHAIN_WHY_FLUSHED: the desync E at s (anchored there) after the walk's flush
    int32_t fin, pad3;            // written last (after a system-scope fence): the record is complete -- the host may
                                  // take the file up while other walks still run (batch.cpp, early resolution)
};
// (CHAIN_WHY_FLUSHHIT: no longer emitted -- the walk takes that flush itself and stops with CHAIN_WHY_FLUSHED)
enum { CHAIN_WHY_NONE = 0, CHAIN_WHY_EVCAP, CHAIN_WHY_END, CHAIN_WHY_PHASE, CHAIN_WHY_TAIL, CHAIN_WHY_NOKSET,
       CHAIN_WHY_CUT, CHAIN_WHY_FLUSH, CHAIN_WHY_BUCKET, CHAIN_WHY_FLUSHHIT, CHAIN_WHY_DEADCAP, CHAIN_WHY_CLOSED,
       CHAIN_WHY_FLUSHED };
// The phase-0 hit map (chain_help): while one file's walk searches tile after tile on its CU, the workgroups whose
// own walks have ended (and the launch's extra ones) map that file's prefix ahead of it -- in the synced state the
// key at p is the true weak sum T(p), whatever the walk does.  One 64-bit word per 32 positions: the map's
// generation (high half) and bit i = "T(32 w + i) is in the table" (low half), written in one store, so that a
// word either carries this launch's generation and its bits or is ignored.  ChainHelp is the file's shared state,
// in device memory, reset by the host before each phase-0 launch.
struct ChainHelp {
    int32_t nseg;    // map segments of CHAIN_MAP_SEG positions over [0, hend) (0: not mapped)
    int32_t claim;   // next segment a helper takes (atomic)
    int32_t live;    // 1 while the file's walk runs (the walk clears it)
    int32_t tiles;   // tiles the walk has searched so far (helpers join files that searched help_tiles)
    int64_t pos;     // the walk's current search start (helpers skip segments behind it)
    int32_t mapped;  // segments mapped (trace)
    int32_t joins;   // helpers that built this file's key set (trace)
    int64_t t_start, t_first;  // wall clock: the walk's start, the first segment mapped ahead of it (trace)
    int64_t t_kset;            // wall-clock ticks spent building this file's key set in helpers (trace)
    int32_t whole;             // segments mapped whole, before the walk reached them (trace)
    int32_t nhelp;             // helpers currently on this file
    int32_t help_tiles;        // tiles the walk searches before helpers join it (A/B switch chain_help_tiles: 1; 4 until
                               // round 5, 4.625 against 4.57 ms for config 4 half, r5m4)
};
constexpr int CHAIN_THREADS = 512;                      // 8 waves (2 per SIMD: 256 VGPRs each)
constexpr int CHAIN_PPT = 32;                            // wide tiles: positions per lane (two halves of 16)
constexpr int64_t CHAIN_TILE = (int64_t)CHAIN_THREADS * CHAIN_PPT;
constexpr int CHAIN_SEGS = 64;                           // blocks a tile may start (B >= 512 when wide)
constexpr int64_t CHAIN_MAP_SEG = 2 * CHAIN_TILE;        // positions per helper claim

struct ChainFile {
    const uint8_t* data;
    int64_t n;
    uint32_t B;
    int32_t C, dl, rem;
    uint32_t kmask;
    const unsigned long long* kslots;  // the chunk index: (key << 32) | (i + 1) per chunk i (launch_chunk_index);
                                       // key presence and buckets both come from it
    const int32_t* table_weak;
    const uint8_t* table_strong;
    const int32_t* aw;                 // the aligned speculation over windows [0, na): weak, digests, chain flags
    const uint8_t* as;
    const uint8_t* flags;
    int64_t na;
    int64_t na_a;                      // phase 0: the speculated prefix's windows (<= na)
    int* abort;                        // phase 0 writes abort_gen here when the file needs no more speculation: done,
                                       // or poisoned by a digest no chunk carries (its phase-1 K1 groups stop)
    rsh_event* ev;
    int32_t ev_cap;
    uint32_t seed;                     // the checksum seed (a window's digest at an unaligned hit)
    ChainOut* out;
    unsigned long long* hmap;          // its map words, positions [0, hend) (null: not mapped)
    int64_t hend;                      // min(na_a B, n - B + 1): the positions a phase-0 search may reach
    const uint8_t* dup;                // per chunk: 1 when another chunk has its weak sum (launch_chunk_index)
};
// Diagnostic: the Generator's K1 over n = 64 k B bytes with per-wave clock stamps summed into d_clk[0] (shader clock
// ticks) and d_clk[1] (100 MHz ticks); the production kernels never stamp.
hipError_t launch_k1_clock(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t dl, uint32_t seed_word,
                           int32_t* d_weak, uint8_t* d_strong, unsigned long long* d_clk, hipStream_t s);
// help (phase 0): the files' ChainHelp array, or null (no map); helpers: extra workgroups beyond nfiles that only
// map; finished walks map too.  abort_gen is also the map's generation.
// timed: the walks read the wall clock for their section timers (scan_trace's report; ChainOut::t_*).
hipError_t launch_chain_advance(const ChainFile* files, uint32_t nfiles, hipStream_t s, int phase = 1,
                                int abort_gen = 0, ChainHelp* help = nullptr, uint32_t helpers = 0, bool timed = false);
// The chunk indexes of many files (slots and dup bytes cleared by the caller; TableEnt as for the probe hashes): the
// index also marks dup[i] = 1 for every chunk i whose weak sum another chunk has, so that the walk decides an aligned
// hit whose chain flag is set without looking the bucket up.
struct ChunkIndexEnt {
    TableEnt t;
    uint8_t* dup;
};
hipError_t launch_chunk_index(const ChunkIndexEnt* ents, uint32_t nfiles, int32_t max_keys, hipStream_t s,
                              bool bg = false);

// splitmix64 counter stream (bench input): byte i = byte (i % 8) of mix(key + (i / 8 + 1) * golden).
hipError_t launch_fill_splitmix(uint8_t* d_out, int64_t n, uint64_t key, int64_t byte_offset, hipStream_t s);

}  // namespace rsh
