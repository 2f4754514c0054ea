// ctx.h -- internals shared by the library's host sources (not part of the C-ABI): device / pinned buffers,
// the rsh_ctx definition, error capture and the one-call-per-context claim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <vector>

#include "device.h"
#include "hit_cache.h"
#include "options.h"
#include "resolver.h"
#include "rsync_hip.h"

namespace rsh {
struct BatchState;  // batch.cpp
void destroy_batch_state(BatchState* b);
hipError_t clear_batch_abort_words(BatchState* b);  // batch.cpp: every file's abort word and map word back to 0
// batch.cpp: the cores this process may use (affinity mask, cgroup quota; option host_cores overrides)
int host_cores();
// The cores one call on this thread may use: host_cores(), or this thread's share of them while a multi-context
// segment call (multi.cpp) runs one member call per context side by side -- each member's MD5 pool, resolver workers
// and copy threads then stay within its share, and the members together within the process's cores.
struct CoreShare {
    static int& value() {
        static thread_local int v = 0;
        return v;
    }
    int saved;
    explicit CoreShare(int cores) : saved(value()) { value() = cores; }
    ~CoreShare() { value() = saved; }
};
inline int call_cores() { return CoreShare::value() > 0 ? std::min(host_cores(), CoreShare::value()) : host_cores(); }
// multi.cpp: whether option fault_inject's bits 0 / 1 apply on this thread (bit 2 limits them to member 1 of a
// multi-context call; tests only)
bool fault_here();
// segment.cpp: one scan's (or pass's) stats added into a call's
void add_scan_stats(rsh_scan_stats* to, const rsh_scan_stats& s);
// The batched scan's resolver threads on this thread's calls: at most this many cores (0: host_cores()).  A segment
// call that digests its files on the other cores meanwhile (segment.cpp) sets it, so that the spinning resolver
// workers and the MD5 pool together stay within the cores (a cgroup quota throttles the whole process past it).
struct WorkerCap {
    static int& value() {
        static thread_local int v = 0;
        return v;
    }
    int saved;
    explicit WorkerCap(int cap) : saved(value()) { value() = cap; }
    ~WorkerCap() { value() = saved; }
};
// batch.cpp: the batched scan's state pre-sized for a segment of nfiles files of n bytes (B, dl) at context creation
hipError_t batch_warm(rsh_ctx* c, int32_t nfiles, int64_t n, int64_t B, int32_t dl);
// batch.cpp: rsh_block_sums_batch_device / rsh_match_scan_batch_device for a caller that holds the context's
// claim (segment.cpp's host-memory forms)
int block_sums_batch_claimed(rsh_ctx* ctx, const rsh_block_job* jobs, int32_t njobs, const uint8_t seed[4]);
int match_scan_batch_claimed(rsh_ctx* ctx, rsh_scan_job* jobs, int32_t njobs, const uint8_t seed[4],
                             rsh_scan_stats* stats);
}  // namespace rsh

namespace rshi {

constexpr int64_t kChunkSize = 8192;        // Sender.java:230 CHUNK_SIZE
constexpr int64_t kDefaultBlock = 8192;     // FileView.java:38 DEFAULT_BLOCK_SIZE
constexpr int32_t kMaxBlockLength = 1 << 17;  // Checksum.java:151
// Speculation launch decision (scan.cpp scan_device, batch.cpp scan_batch): when the first kLeadWindows
// aligned source windows all carry their chunk's weak sum, a run of aligned matches is likely: the
// speculation is launched at once and the resolver waits for it instead of taking head-mode steps.
constexpr int64_t kLeadWindows = 32;

// Option scan_trace = 1: one stderr line per buffer allocation (where a call's first-use costs go)
inline void trace_alloc(const char* what, size_t n, std::chrono::steady_clock::time_point t0) {
    if (rsh::opt(rsh::OPT_SCAN_TRACE) == 1)
        fprintf(stderr, "[rsh] %-10s %10zu %9.3f ms\n", what, n,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipMalloc(&p, n ? n : 1);
        if (e == hipSuccess) cap = n;
        trace_alloc("dev_alloc", n, t0);
        return e;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Page-locked host staging (true async D2H).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        // small buffers grow geometrically: a round-trip buffer that creeps up by a few entries per call
        // would otherwise pay a pinned allocation (~0.1-1 ms) every time
        if (n < (64u << 20)) n = std::max<size_t>({n, std::min<size_t>(2 * cap, 64u << 20), 64u << 10});
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        trace_alloc("pin_alloc", n, t0);
        return e;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

inline uint32_t seed_word(const uint8_t seed[4]) {
    return (uint32_t)seed[0] | ((uint32_t)seed[1] << 8) | ((uint32_t)seed[2] << 16) | ((uint32_t)seed[3] << 24);
}

inline uint32_t pow2_at_least(uint64_t v) {
    uint32_t p = 64;
    while (p < v) p <<= 1;
    return p;
}

inline double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// rsh_match_scan_tiled: default tile (the device holds one tile + a 16 B halo of the source at a time)
constexpr int64_t kDefaultTile = 4LL << 30;

// Option scan_trace = 1: one stderr line per resolver round trip (diagnostics).
struct CallTrace {
    const char* what;
    int64_t arg;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    static bool on() { return rsh::opt(rsh::OPT_SCAN_TRACE) != 0; }
    CallTrace(const char* w, int64_t a) : what(w), arg(a) {}
    ~CallTrace() {
        if (on()) fprintf(stderr, "[rsh] %-10s %10lld %9.3f ms\n", what, (long long)arg, ms_since(t0));
    }
};

}  // namespace rshi
using namespace rshi;
using rsh::HitCache;

struct rsh_ctx {
    int device = 0;
    int n_cu = 256;  // compute units (the chain walk's helper workgroups fill the ones its files leave idle)
    hipStream_t stream = nullptr;
    DevBuf data, weak, strong;                   // host-input staging
    DevBuf src_weak, src_strong, flags;          // aligned speculation over the source
    // phase-shifted speculation over [s0, n) (chains at kB + delta): two buffer sets used in turn, so that a
    // launch never writes the sums (or their host copies) of the launch it replaces while that one drains
    DevBuf ph_weak[2], ph_strong[2];
    DevBuf segs;                                 // segmented K1 descriptors (prefix + phase speculation)
    DevBuf slots, dslots, out, first, haw, partials, bucket;
    DevBuf seg_data, seg_tab;                    // rsh_*_batch (segment.cpp): a pass's files and tables / sums
    DevBuf rcv[2], rcv_ops[2];                   // rsh_receiver_combine_batch: two pass buffers and their gather ops
    DevBuf prep_dev;                             // the stamped launches' counters and the prep launch's scratch
    DevBuf fc_dev;                               // the batched flush chain's gathered sums and bytes (flush_probe)
    hipStream_t aux = nullptr;                   // the aligned speculation
    hipStream_t phase = nullptr;                 // the phase-shifted speculation (beside a prefix speculation)
    hipEvent_t ev_in = nullptr, ev_tab = nullptr, ev_spec = nullptr;
    hipEvent_t ev_phase[2] = {nullptr, nullptr};  // set i's last phase launch and its downloads are done
    hipEvent_t ev_prep = nullptr;   // the scan's table and sample work on the context stream (A/B ordering)
    hipEvent_t ev_flags = nullptr;  // batched speculation: its chain flags are on the host (before its sums)
    hipEvent_t ev_k1a = nullptr, ev_k1b = nullptr;  // timing: the aligned speculation's K1 (stats)
    hipEvent_t ev_gen_a = nullptr, ev_gen_b = nullptr;  // timing: rsh_block_sums_device's K1 (rsh_debug_kernel_ms)
    bool gen_timed = false;                             // ... recorded by the last rsh_block_sums_device
    bool spec_timed = false;                            // ev_k1a / ev_k1b belong to the last scan's speculation
    hipEvent_t ev_rs_tail = nullptr;  // scan_spec_queue: the end of a scan's work on aux (see spec_buffers_free)
    hipEvent_t ev_pha[2] = {nullptr, nullptr}, ev_phb[2] = {nullptr, nullptr};  // timing: set i's phase K1 (stats)
    int ph_set = 0;  // the buffer set of the latest phase launch
    PinnedBuf h_weak, h_strong, h_aw, h_as, h_fl;
    PinnedBuf h_pw[2], h_ps[2];  // the phase-shifted speculation's sums (host copies), per set
    PinnedBuf h_segs;      // staging of the segmented K1 descriptors
    PinnedBuf h_lead;      // T(kB) of the first aligned windows (the speculation launch decision)
    // resolver round trips: the small kernels read their inputs from and write their outputs to pinned
    // host memory directly (no staging copies); the probe result and digest windows come back by copy
    PinnedBuf h_pos, h_out, h_iv, h_tiles, h_keys, h_first, h_win, h_ptiles, h_psegs;
    PinnedBuf h_hit;  // after a probe hit: T(p) (bytes 0..3) and the window at p (from byte 16)
    PinnedBuf h_win0;    // window 0 of the current scan (its digest is computed on a host thread)
    PinnedBuf h_pend;    // the prefix end's window sums (launched with the phase guess's first probe)
    PinnedBuf h_bucket;  // after a probe hit: {count, key, chunk indices} of the key that hit
    PinnedBuf h_files;   // the scan's rsh::ScanFile (a batch of one for the probe / gather kernels)
    PinnedBuf h_stage;   // file ingest ring (ingest.cpp); never shared with the scan's buffers
    PinnedBuf h_rcv_ops[2];  // rsh_receiver_combine_batch: the gather ops of a pass, staged
    PinnedBuf h_prep;        // the prep launch's outputs (scan_spec_queue)
    PinnedBuf h_stamps;      // the stamped launches' stamps, one 64-B line each
    PinnedBuf h_fgw, h_fjobs, h_fout;  // flush_probe: the chain's gather list, its job, its outputs
    uint64_t first_used = 0;    // probe result slots handed out (see HipBackend::first_hit)
    // device, uncached, 256 B: the speculation launch of generation g stops once abort_word[0] holds g;
    // a phase-shifted speculation polls abort_word[kPhaseWord] (its own 64-B line)
    int* abort_word = nullptr;
    static constexpr int kPhaseWord = 16;
    int gen = 0;
    // The next launch generation.  Launches compare their abort word with their generation for equality, and a word
    // keeps the last generation it was set to: after 2^31 launches the counter would come back to a value a word still
    // holds and a fresh launch would stop itself (or a walk trust a stale hit-map word, which carries its launch's
    // generation).  So before it wraps, the device drains, every abort and map word goes back to 0 and the count
    // restarts at 1 (once per ~2 billion launches; test_generation_wrap).
    int next_gen();
    static constexpr int kGenWrapAt = 0x7FFFFF00;  // below INT32_MAX by more than one call's launches
    bool spec_dl_pending = false;  // the last speculation's sums download (aux) may still read src_weak / src_strong
    int stamp_seq = 0;             // values of the stamped launches (scan.cpp prep_ensure)
    // the next stamp value, 1..INT32_MAX and wrapping: a stamp is compared for equality, and 0 is a pinned word's
    // initial value (a context that lives for billions of probes must not overflow the counter)
    int next_stamp() {
        stamp_seq = stamp_seq == INT32_MAX ? 1 : stamp_seq + 1;
        return stamp_seq;
    }
    std::vector<rsh_event> last_ev;  // kept when the caller's event buffer was too small
    std::atomic<bool> busy{false};   // the staging buffers and last_ev serve one call at a time
    rsh::BatchState* batch = nullptr;  // buffers of the batched (multi-file) entry points, on first use
    ~rsh_ctx() {
        if (batch) rsh::destroy_batch_state(batch);
        for (DevBuf* b : {&data, &weak, &strong, &src_weak, &src_strong, &flags, &ph_weak[0], &ph_strong[0],
                          &ph_weak[1], &ph_strong[1], &slots, &dslots,
                          &out, &first, &haw, &partials, &bucket, &seg_data, &seg_tab,
                          &rcv[0], &rcv[1], &rcv_ops[0], &rcv_ops[1], &prep_dev, &fc_dev})
            b->release();
        for (PinnedBuf* b : {&h_weak, &h_strong, &h_aw, &h_as, &h_fl, &h_pw[0], &h_ps[0], &h_pw[1], &h_ps[1], &h_lead, &h_pos, &h_out, &h_iv,
                             &h_tiles, &h_keys, &h_first, &h_win, &h_ptiles, &h_psegs, &h_hit, &h_win0, &h_pend, &h_bucket, &h_files,
                             &h_stage, &h_rcv_ops[0], &h_rcv_ops[1], &h_prep, &h_stamps, &h_fgw, &h_fjobs, &h_fout})
            b->release();
        if (abort_word) (void)hipFree(abort_word);
        if (ev_in) (void)hipEventDestroy(ev_in);
        if (ev_tab) (void)hipEventDestroy(ev_tab);
        if (ev_spec) (void)hipEventDestroy(ev_spec);
        for (hipEvent_t e : {ev_phase[0], ev_phase[1], ev_pha[0], ev_pha[1], ev_phb[0], ev_phb[1]})
            if (e) (void)hipEventDestroy(e);
        if (ev_flags) (void)hipEventDestroy(ev_flags);
        if (ev_prep) (void)hipEventDestroy(ev_prep);
        for (hipEvent_t e : {ev_k1a, ev_k1b, ev_gen_a, ev_gen_b, ev_rs_tail})
            if (e) (void)hipEventDestroy(e);
        if (aux) (void)hipStreamDestroy(aux);
        if (phase) (void)hipStreamDestroy(phase);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// Last HIP failure of the calling thread (rsh_last_error): error text and the source line.
inline thread_local char g_last_err[256] = "";
inline void note_error(hipError_t e, int line, const char* file = "capi.cpp") {
    snprintf(g_last_err, sizeof(g_last_err), "%s (%s:%d)", hipGetErrorString(e), file, line);
}

#define RSH_HIP(call)                                   \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) {                         \
            note_error(e_, __LINE__, __FILE__);         \
            return RSH_E_DEVICE;                        \
        }                                               \
    } while (0)

namespace rshi {

// Claims a context for one call that uses its buffers; a second thread gets RSH_E_BUSY instead of
// racing on them (one rsh_ctx per calling thread, rsync_hip.h).
struct CtxClaim {
    rsh_ctx* c;
    bool held;
    explicit CtxClaim(rsh_ctx* ctx) : c(ctx), held(!ctx->busy.exchange(true, std::memory_order_acquire)) {}
    ~CtxClaim() {
        if (held) c->busy.store(false, std::memory_order_release);
    }
};

#define RSH_CLAIM(ctx)                                                                   \
    CtxClaim claim_(ctx);                                                                \
    if (!claim_.held) {                                                                  \
        snprintf(g_last_err, sizeof(g_last_err), "context in use by another thread");   \
        return RSH_E_BUSY;                                                               \
    }

// Header consistency for the Generator side (3-arg ctor semantics, Checksum.java:94-113).
inline int check_generator_header(int64_t n, const rsh_header* h) {
    if (!h || n < 0) return RSH_E_INVAL;
    if (h->block_length == 0) return (h->chunk_count == 0) ? RSH_OK : RSH_E_INVAL;
    if (h->block_length < 0 || h->digest_length < 0 || h->digest_length > 16) return RSH_E_INVAL;
    const int64_t B = h->block_length;
    const int64_t rem = n % B;
    const int64_t cc = n / B + (rem > 0 ? 1 : 0);
    if (cc > 2147483647LL) return RSH_E_OVERFLOW;
    if (cc != h->chunk_count || rem != h->remainder) return RSH_E_INVAL;
    return RSH_OK;
}

// Sender.skipMatchSendData (Sender.java:1386-1399): one sendDataFrom per 8 KiB FileView window.
inline void skip_events(int64_t n, rsh::ResolveResult* r) {
    for (int64_t s = 0; s < n; s += kDefaultBlock)
        r->ev.push_back(rsh_event{s, std::min<int64_t>(kDefaultBlock, n - s), RSH_EV_LITERAL, 0, 0, 0});
    r->literal = n;
}

// scan.cpp: a new context's warm-up (code objects, the copy paths, a config-5 file's scan buffers: rsh_ctx_create)
hipError_t ctx_warm(rsh_ctx* c);
// scan.cpp: the device-resident Sender scan (everything but the whole-file MD5) and the event hand-out.
int scan_device(rsh_ctx* c, const uint8_t* d_src, int64_t n, const rsh_header* h, const int32_t* d_weak,
                const uint8_t* d_strong, const int32_t* host_weak, const uint8_t* host_strong, const uint8_t seed[4],
                rsh::ResolveResult* res);
int emit_events(rsh_ctx* c, rsh::ResolveResult& r, rsh_event* ev, int64_t cap, int64_t* n_ev);
// scan.cpp: the scan with HBM holding one tile of the source at a time (fill copies source bytes to HBM).
int scan_tiled(rsh_ctx* c, const std::function<hipError_t(uint8_t*, int64_t, int64_t)>& fill, int64_t n,
               const rsh_header* h, const int32_t* d_weak, const uint8_t* d_strong, const int32_t* host_weak,
               const uint8_t* host_strong, const uint8_t seed[4], int64_t tile_bytes, rsh::ResolveResult* res);

// Primes the resolver's table with the buckets the device computed with a probe (device.h HIT_BUCKET_INTS
// layout, copied to the host): the first hit's, and each listed hit's when it fits LISTED_IDX entries.
inline void prime_from_probe(rsh::ChunkTable& t, const rsh::ProbeOut& o, const int32_t* b) {
    t.prime_clear();
    if (o.first == ~0ull) return;
    if (b[0] <= rsh::HIT_BUCKET_CAP) t.prime(b[1], b + 2, b[0]);
    if (o.count > (unsigned long long)rsh::PROBE_HITS_CAP) return;
    const int32_t* lb = b + 2 + rsh::HIT_BUCKET_CAP;
    for (unsigned long long j = 0; j < o.count; ++j) {
        const int32_t* e = lb + (1 + rsh::LISTED_IDX) * j;
        if (e[0] <= rsh::LISTED_IDX) t.prime((int32_t)o.key[j], e + 1, e[0]);
    }
}

}  // namespace rshi
