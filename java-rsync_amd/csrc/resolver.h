// resolver.h -- the sequential part of Sender.sendMatchesAndData (Sender.java:1235-1327), driven by
// sparse events that the device computes in bulk.
//
// The Java loop is byte-serial and history dependent (preferred index, the cached localChunkMd5sum
// declared outside the loop, the rolling sum that is not recomputed after a FileView flush).  The
// resolver reproduces it exactly while touching only O(events) positions:
//   * aligned chains: the device computes the source's own block sums (same B, dl as the basis
//     table) and a flag per k "source window k has chunk k's weak key and digest"; a run of flags
//     starting where the preferred index equals k is a run of matches (no per-byte work);
//   * otherwise the next candidate event is the first position whose rolling key R(p) = T(p) + E(p)
//     hits the table (or, once the cached digest D is stale, hits a chunk whose digest is D); the
//     device answers that with one range probe per state change;
//   * flushes (FileView.isFull) happen at mark + 9B exactly and are applied in closed form, including
//     the desync E they introduce (E_lo constant, E_hi += E_lo per full-window step).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "rsync_hip.h"

namespace rsh {

// Host time in the table operations of the calling thread (RSH_SCAN_TRACE diagnostics).
struct HostTimes {
    double bucket_ms = 0, sort_ms = 0, dkeys_ms = 0, md5_ms = 0;
};
HostTimes& host_times();

// Host view of the received chunk table (Checksum + Multimap, Checksum.java:156-276).
struct ChunkTable {
    int32_t chunk_count = 0;
    int32_t block_length = 0;
    int32_t remainder = 0;
    int32_t digest_length = 0;
    const int32_t* weak = nullptr;   // chunk_count, receive order
    const uint8_t* strong = nullptr; // chunk_count * digest_length

    // Ascending chunk indices whose weak key is `key` (a Multimap bucket, in insertion order); valid
    // until the next call.  The first kScanLookups lookups are linear scans of `weak`; then the table is
    // indexed once (a chained hash over a private copy of the keys, built in one pass) and lookups walk
    // one chain.  A scan that poisons early (quirk B) needs a handful of lookups and never builds it.
    const int32_t* bucket(int32_t key, int32_t* size);
    void build();  // index now
    bool indexed() const { return indexed_; }
    double sort_ms = 0;  // time spent in build()
    int32_t chunk_length(int32_t idx) const {  // Checksum.java:197-203
        return (idx == chunk_count - 1 && remainder > 0) ? remainder : block_length;
    }
    // Distinct weak keys of the chunks whose digest equals d (the only ones a stale digest can match).
    void keys_with_digest(const uint8_t* d, std::vector<int32_t>* keys) const;

    static constexpr int kScanLookups = 2;
    // The bucket of `key` computed elsewhere (the device, in the round trip that found a probe hit):
    // idx ascending.  The next bucket(key) returns it without touching the table.
    // The device computes buckets with each probe (the first hit's, and those of the listed hits): they
    // stand in for lookups until the next probe (prime_clear).
    void prime_clear() { primed_n_ = 0; }
    void prime(int32_t key, const int32_t* idx, int32_t count) {
        if (primed_n_ == (int)primed_.size()) primed_.emplace_back();
        Primed& e = primed_[(size_t)primed_n_++];
        e.key = key;
        e.idx.assign(idx, idx + count);
        std::sort(e.idx.begin(), e.idx.end());
    }

  private:
    struct Primed {
        int32_t key;
        std::vector<int32_t> idx;
    };
    std::vector<Primed> primed_;
    int primed_n_ = 0;
    bool indexed_ = false;
    int scan_lookups_ = 0;
    // chained hash index: head_[hash(key)] = smallest chunk index with that hash, next_[i] = the next
    // larger one (chains ascend, so a bucket comes out in Multimap insertion order)
    uint32_t index_mask_ = 0;
    std::vector<int32_t> head_, next_;
    std::vector<int32_t> weak_copy_;  // the received table usually sits in pinned host memory
    std::vector<int32_t> scratch_;
};

// One probe interval: positions [a, b) with the key R(p) = T(p) + E(p),
// E(p) = (e_lo, e_hi + e_lo * (min(p, n-B) - min(anchor, n-B))) mod 2^16.
struct ProbeInterval {
    int64_t a, b, anchor;
    uint32_t e_lo, e_hi;
};

// The batched flush chain (resolver.cpp step 2; FileView.isFull at mark + 9B, Sender.java:1294-1310): flushes at
// f_i = f + 10 B i (i < K), flush i from the rolling value R_i at f_i -- R_0 = T(f) + E with E = (el, eh) at f,
// R_{i+1} = T(f_{i+1}) + E_i(f_{i+1}) -- and E_i = R2_i - T(f_i + B) after it (quirk A: the Java code subtracts x_f
// with the full window, slides by B and keeps rolling the old value).  Step i opens the interval
// [s2_i, min(s2_i + 9B, last) + 1) = [f_i + B, ...) with desync (elo_i, ehi_i) anchored at s2_i; a step whose s2 is
// past `last` ends the chain.
struct FlushChain {
    int64_t f = 0, K = 0, B = 0, n = 0, last = 0;
    uint32_t el = 0, eh = 0;
};
struct FlushStep {
    int64_t s2;
    uint32_t elo, ehi;
};
// the positions the chain reads: T at f_i and f_i + B (tpos, 2K), the bytes at f_i and f_i + 2B - 1 (bpos, 2K)
void flush_positions(const FlushChain& q, std::vector<int64_t>* tpos, std::vector<int64_t>* bpos);
// the steps' s2 and their intervals' bounds (E left 0): what does not depend on the sums
void flush_intervals(const FlushChain& q, std::vector<FlushStep>* steps, std::vector<ProbeInterval>* ivs);
// the chain itself from the gathered sums and bytes: steps and intervals with their E
void flush_chain_host(const FlushChain& q, const int32_t* tv, const uint8_t* bv, std::vector<FlushStep>* steps,
                      std::vector<ProbeInterval>* ivs);

// Speculated sums of the source windows at s0 + kB, k in [0, count) (a phase-shifted speculation: the
// source's own block sums from s0 on, with the received header's B and dl).  w[k] = T(s0 + kB) over
// min(B, n - s0 - kB) bytes, st + k * dl = that window's MD5 || seed, cut / zero-padded to dl bytes.
struct PhaseView {
    int64_t s0 = 0, count = 0;
    const int32_t* w = nullptr;
    const uint8_t* st = nullptr;
};

// Device (or test) services used by the resolver.  Positions are source file offsets.
class ScanBackend {
  public:
    virtual ~ScanBackend() {}
    // Shifted chains (Sender.java:1282-1287: after a match the scan jumps a whole window, so consecutive
    // matches chain at any phase, not only at kB).  phase_hint(s): a match just left the scan synced at a
    // non-aligned s; the backend may start a speculation over [s, n).  phase_sums(s, wait, v): sums of a
    // speculation whose windows include s, if one has landed (wait: block until an in-flight one that
    // covers s lands).  false = none; the resolver then takes the generic path (same answer).
    virtual void phase_hint(int64_t s) { (void)s; }
    virtual bool phase_sums(int64_t s, bool wait, PhaseView* v) {
        (void)s, (void)wait, (void)v;
        return false;
    }
    // Aligned speculation over the source: window k = [kB, min(kB + B, n)), k < aligned_count().
    virtual int64_t aligned_count() = 0;
    // Windows whose chain flag is known (the flags may land before the aligned sums they are computed from).
    virtual int64_t flags_count() { return aligned_count(); }
    virtual const int32_t* aligned_weak() = 0;
    virtual const uint8_t* aligned_strong() = 0;  // digest_length bytes per window
    virtual const uint8_t* chain_flags() = 0;     // min(aligned_count, chunk_count) entries
    virtual void weak_many(const int64_t* pos, int64_t count, int32_t* out) = 0;  // T(p) over min(B, n-p) bytes
    virtual void bytes_many(const int64_t* pos, int64_t count, uint8_t* out) = 0;
    virtual void md5_at(int64_t p, uint8_t out[16]) = 0;  // MD5(x[p, p + min(B, n-p)) || seed)
    // Smallest p over all intervals whose key is in the key set (keys == nullptr: the whole chunk
    // table); -1 if none.
    virtual int64_t first_hit(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys) = 0;
    // Upper bound on the flush intervals one batched probe may cover (max_batch_at: for a batch whose first
    // flush point is f -- a tiled backend keeps the batch inside its resident tile).
    virtual int64_t max_batch() { return 4096; }
    virtual int64_t max_batch_at(int64_t f) {
        (void)f;
        return max_batch();
    }
    // Whether one device round may read from positions a through b (a <= b): a tiled backend answers each round
    // from the tile holding its first position, and tiles only advance, so a probe at a and a flush chain at b go
    // out together only when both lie in one tile; otherwise the resolver asks in two rounds, in order.
    virtual bool one_round(int64_t a, int64_t b) {
        (void)a, (void)b;
        return true;
    }
    // Source bytes the backend's device work read for this scan (rsh_scan_stats::device_bytes).
    int64_t bytes_read = 0;
    static int64_t probe_bytes(const ProbeInterval* iv, int64_t count, int64_t B) {
        int64_t b = 0;
        for (int64_t i = 0; i < count; ++i) b += (iv[i].b - iv[i].a) + B - 1;
        return b;
    }

    // The batched flush chain's gather: weak sums at tpos and bytes at bpos, in one device round trip where
    // the backend can.
    virtual void flush_gather(const int64_t* tpos, int64_t nt, int32_t* tv, const int64_t* bpos, int64_t nb,
                              uint8_t* bv) {
        weak_many(tpos, nt, tv);
        bytes_many(bpos, nb, bv);
    }

    // The batched flush chain and one probe: the intervals pre[0, npre) (E known; the interval the scan is in),
    // then the chain's intervals.  Fills *steps and *ivs as flush_chain_host and returns the first hit over
    // pre + ivs (-1: none).  Default: flush_gather, the chain on the host, first_hit (two round trips); the GPU
    // backends gather, chain (device.h launch_flush_chain) and probe in one.
    virtual int64_t flush_probe(const ProbeInterval* pre, int64_t npre, const FlushChain& q,
                                std::vector<FlushStep>* steps, std::vector<ProbeInterval>* ivs,
                                const std::vector<int32_t>* keys);

    int32_t weak_at(int64_t p) {
        int32_t r;
        weak_many(&p, 1, &r);
        return r;
    }
    uint8_t byte_at(int64_t p) {
        uint8_t r;
        bytes_many(&p, 1, &r);
        return r;
    }
};

struct ResolveResult {
    std::vector<rsh_event> ev;
    int64_t literal = 0;
    int64_t matched = 0;
    rsh_scan_stats stats{};
};

// The Sender's state between resolver steps (Sender.java:1241-1249 locals + FileView mark/start).
// E = R - T is kept as its value at `anchor` (quirk A).
struct ResolveState {
    int64_t s = 0, m = 0;
    int32_t pref = 0;
    uint32_t elo = 0, ehi = 0;
    int64_t anchor = 0;
    bool md5c_valid = false;  // localChunkMd5sum != null (Sender.java:1248)
    std::vector<uint8_t> md5c;  // digest_length bytes: Arrays.copyOf(MD5, dl), zero past 16 (:1262)
    std::vector<int32_t> dkeys;  // weak keys of the chunks whose digest is md5c
    bool dkeys_ready = false;
    int64_t batch = 1;  // flush intervals speculated per batched probe
    bool done = false;
    // handed over by the device chain walk: no candidate event in [clear_from, clear_to] -- its search reached the
    // flush point -- so the first step (2) from s == clear_from needs no probe (consumed by that step)
    int64_t clear_from = -1, clear_to = -1;
};

// n > 0 and h->block_length > 0 (skipMatchSendData / empty sources are handled by the caller).
// Runs the scan from *state to the end (returns true) or until yield() -- asked between two steps --
// returns true (returns false; call again with the same state and result to resume).  The backend's
// aligned speculation is re-read on every call, so a scan can start before it exists.
bool resolve_run(int64_t n, ChunkTable& table, ScanBackend& be, ResolveState* state, ResolveResult* out,
                 const std::function<bool()>& yield);
void resolve_scan(int64_t n, ChunkTable& table, ScanBackend& be, ResolveResult* out);

}  // namespace rsh
