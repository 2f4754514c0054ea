// batch.h -- the batched Sender scan's shared state (not part of the C-ABI): the per-context BatchState, a file's
// resolver (FileScan: its table, state and BatchBackend), the requests its fiber posts (Req) and the rounds that answer
// them (Batch).  batch.cpp plans a segment's scan and drives its chain walks (scan_batch); batch_pool.cpp runs the
// resolvers that are left as fibers on a pool of worker threads and answers their device questions one round at a
// time (run_resolvers, serve_round).
//
// The fiber scheduler's invariants (match_scan_batch_claimed; Batch, FileScan, fiber_main):
//  1. Ownership.  Live file i belongs to worker i % W for the whole scan; only that worker's thread ever switches
//     into its fiber, so a FileScan's resolver state (table, ResolveState, BatchBackend) is touched by one thread
//     at a time, without locks.  The coordinator reads a FileScan (req, pending, done) and writes its answer only
//     while every worker is idle (2).
//  2. Rounds.  A round starts when the coordinator bumps `gen` under `mu` and ends when `idle == nworkers`.  In
//     between the coordinator touches no FileScan; the workers touch nothing shared but their own slots of
//     busy_ms / max_fiber_ms / times and (under `mu`) `idle`, `nworkers`.  The release of `mu` (or the
//     acquire-load of `gen` / `idle` in spin_wait, re-checked under `mu`) orders a round's fiber writes before
//     the coordinator's reads and the coordinator's answers before the next round's fiber reads.
//  3. Requests.  A fiber posts at most one request and then switches back to its worker (Batch::post); `pending`
//     stays set until the worker resumes it in a later round, so every request is answered exactly once.  A WAIT
//     request is resumed only once `landed` is set; the worker keeps such a file (it does not leave while any of
//     its files is not done), so the coordinator never waits on a file no worker will run.
//  4. Termination.  The coordinator ends the scan in the round where no file is pending and every worker is idle
//     or gone: every fiber has returned (done) and no fiber stack is live.  It sets `quit`, and the workers exit
//     on their next wake-up; they are detached and keep only `bp` (a shared_ptr) alive, never FileScan or the
//     stacks, which the next scan reuses.
//  5. Device work and errors.  Only the coordinator launches device work or synchronises streams during the
//     rounds (serve_round, the speculation's launch and cancellation); a fiber's device question is answered from
//     host memory the round's synchronisation made valid.  A failed round records the first HIP error and keeps
//     serving (the resolvers finish on whatever the round left), and the scan returns RSH_E_DEVICE after the
//     rounds: no fiber is ever left suspended and no worker blocked.
//  6. Cores.  W <= min(live files, host cores - 1 when waiters spin, kMaxWorkers); the spinning waiters leave one
//     core for the coordinator, and rsh_match_scan_batch caps the workers (WorkerCap) so that the multi-buffer
//     MD5 pool running beside the scan does not oversubscribe the process's cores.
#pragma once
#include <sched.h>
#include <ucontext.h>

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#include <immintrin.h>

#include "ctx.h"
#include "host_md5.h"
#include "options.h"
#include "resolver.h"

namespace rsh {

// A few persistent host threads for a batched call's bulk host copies (the events back to the callers' buffers):
// threads created per call paid a fresh stack mapping each (~30 us; glibc caches only 40 MiB of stacks), the first call
// for all of them.  run(n, f) calls f(0 .. n-1) on the pool and the calling thread, and returns when all are done.
struct HostPool {
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::vector<std::thread> th;
    const std::function<void(int)>* job = nullptr;
    int njobs = 0, next = 0, done = 0;
    uint64_t gen = 0;
    bool quit = false;
    void ensure(int n) {
        while ((int)th.size() < n) th.emplace_back([this] { work(); });
    }
    void work() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> l(mu);
        for (;;) {
            cv_work.wait(l, [&] { return quit || gen != seen; });
            if (quit) return;
            seen = gen;
            while (next < njobs) {
                const int i = next++;
                l.unlock();
                (*job)(i);
                l.lock();
                if (++done == njobs) cv_done.notify_one();
            }
        }
    }
    void run(int n, const std::function<void(int)>& f) {
        if (n <= 0) return;
        std::unique_lock<std::mutex> l(mu);
        job = &f;
        njobs = n, next = 0, done = 0;
        ++gen;
        cv_work.notify_all();
        while (next < njobs) {  // the caller takes part
            const int i = next++;
            l.unlock();
            f(i);
            l.lock();
            ++done;
        }
        cv_done.wait(l, [&] { return done == njobs; });
        job = nullptr;
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> l(mu);
            quit = true;
        }
        cv_work.notify_all();
        for (std::thread& t : th) t.join();
    }
};

struct BatchState {
    HostPool pool;  // the events' copies (scan_batch)
    // Generator batch
    DevBuf g_groups, g_lanes, g_plans, k1_plans;  // K1 groups are expanded on the device from per-file plans
    // Sender batch: device
    DevBuf slots, dslots, src_weak, src_strong, flags, haw, partials, bucket, first, k1_groups, k1_lanes;
    DevBuf d_probe;  // a large probe's descriptors (files, intervals, tiles, partial tiles) in device memory
    DevBuf fc_dev;   // FCHAIN rounds: the chains' gathered sums and bytes
    PinnedBuf h_fgw, h_fjobs, h_fout;  // ... their gather lists, chain jobs and chain outputs
    PinnedBuf h_early;  // early resolution: one file's copies and its probe hash entry
    PinnedBuf h_rcp;    // a round's answer copies (serve_round)
    // Sender batch: pinned host (read or written by the kernels directly)
    PinnedBuf h_weak, h_strong, h_aw, h_as, h_fl, h_files, h_hit, h_win0, h_bucket, h_first, h_iv, h_tiles, h_segs,
        h_ptiles, h_req, h_gw, h_gb, h_ow, h_ob, h_win, h_copies, h_tabents, h_flagents, h_flagents_a, h_dkeys, h_ccopies,
        h_lead;
    // device, uncached: one abort word per file of the batch; the speculation's groups of file f stop once
    // file_abort[f] holds the scan's generation (written by the coordinator when f's resolver finishes)
    int* file_abort = nullptr;
    int64_t file_abort_cap = 0;
    // Generator batch: its launch descriptors, staged in pinned memory so that the upload is asynchronous
    // (a pageable copy blocks the host while the device idles); ev_gcopy guards the staging buffers' reuse
    PinnedBuf h_ggroups, h_glanes;
    hipEvent_t ev_gcopy = nullptr;
    bool gcopy_pending = false;
    // the same for the Sender's speculation launch (uploaded on the aux stream from the coordinator thread)
    PinnedBuf h_sgroups, h_slanes;
    hipEvent_t ev_scopy = nullptr;
    bool scopy_pending = false;
    // the chain walk (options.h batch_chain): chunk indexes, descriptors, results and events (pinned), and the
    // speculation's flags kernel done on the aux stream (the walk reads the device flags and sums)
    DevBuf kslots;  // the chunk indexes' slots (8 B each), then one duplicate byte per chunk (launch_chunk_index)
    PinnedBuf h_kents, h_chain, h_chain_out, h_chain_ev;
    // the phase-0 hit map (device.h ChainHelp): the files' shared map state (reset from pinned staging before each
    // launch) and the map words (generation-tagged: zeroed once when allocated, never cleared between scans)
    DevBuf chain_help, chain_map;
    PinnedBuf h_chain_help;
    std::vector<std::unique_ptr<char[]>> fiber_stacks;  // the resolver fibers' stacks (batch.cpp workers)
    hipEvent_t ev_fk = nullptr;
    hipEvent_t ev_sync = nullptr;  // spin_sync: the latency-path waits poll an event instead of blocking
    hipEvent_t ev_ch0 = nullptr, ev_ch1 = nullptr;  // around the walk (trace)
    hipEvent_t ev_fa = nullptr, ev_wa = nullptr;    // two-phase walk: prefix flags done, phase-0 walk done
    hipError_t ensure_file_abort(int64_t nf) {
        if (nf <= file_abort_cap) return hipSuccess;
        if (file_abort) (void)hipFree(file_abort);
        file_abort = nullptr;
        file_abort_cap = 0;
        const int64_t cap = std::max<int64_t>(nf, 256);
        hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&file_abort), (size_t)cap * 4,
                                             hipDeviceMallocUncached);
        if (e == hipSuccess) e = hipMemset(file_abort, 0, (size_t)cap * 4);  // generations start at 1
        if (e == hipSuccess) file_abort_cap = cap;
        return e;
    }
    ~BatchState() {
        if (file_abort) (void)hipFree(file_abort);
        if (ev_gcopy) {
            if (gcopy_pending) (void)hipEventSynchronize(ev_gcopy);
            (void)hipEventDestroy(ev_gcopy);
        }
        if (ev_scopy) {
            if (scopy_pending) (void)hipEventSynchronize(ev_scopy);
            (void)hipEventDestroy(ev_scopy);
        }
        for (hipEvent_t e : {ev_fk, ev_ch0, ev_ch1, ev_fa, ev_wa, ev_sync})
            if (e) (void)hipEventDestroy(e);
        kslots.release();
        for (PinnedBuf* b : {&h_kents, &h_chain, &h_chain_out, &h_chain_ev, &h_chain_help}) b->release();
        chain_help.release();
        chain_map.release();
        h_ggroups.release();
        h_glanes.release();
        h_sgroups.release();
        h_slanes.release();
        for (DevBuf* b : {&d_probe, &fc_dev, &g_groups, &g_lanes, &g_plans, &k1_plans, &slots, &dslots, &src_weak, &src_strong, &flags, &haw, &partials, &bucket,
                          &first, &k1_groups, &k1_lanes})
            b->release();
        for (PinnedBuf* b : {&h_weak, &h_strong, &h_aw, &h_as, &h_fl, &h_files, &h_hit, &h_win0, &h_bucket, &h_first,
                             &h_iv, &h_tiles, &h_segs, &h_ptiles, &h_req, &h_gw, &h_gb, &h_ow, &h_ob, &h_win, &h_copies,
                             &h_tabents, &h_flagents, &h_flagents_a, &h_dkeys, &h_ccopies, &h_lead, &h_fgw, &h_fjobs,
                             &h_fout, &h_early, &h_rcp})
            b->release();
    }
};
// BatchState::kslots: the slots of tns chunk-index entries, then tw duplicate bytes (one per chunk)
inline size_t kslots_bytes(int64_t tns, int64_t tw) { return (size_t)tns * 8 + (size_t)tw + 8; }
inline uint8_t* kslots_dup(BatchState* S, int64_t tns) {
    return reinterpret_cast<uint8_t*>(S->kslots.as<unsigned long long>() + tns);
}

namespace batch {

constexpr int32_t kMaxLive = 256;     // files resolved concurrently (one host thread each)
constexpr int kDeferRounds = 2;       // rounds in head mode before the speculation is launched
constexpr int32_t kMaxWorkers = 32;   // host threads running the resolvers
constexpr size_t kFiberStack = 512 * 1024;
constexpr int32_t kEagerSortChunks = 1 << 16;  // tables up to this size are sorted before the first round
constexpr int64_t kPad = 16;
constexpr int64_t kWaveSlots = 2 * 4 * 256;  // the chip's K1 wave slots (2 waves per SIMD, 4 SIMDs, 256 CUs)
constexpr size_t kProbeUpload = 2048;  // probes with more tiles read their descriptors from device memory
// events one file's chain walk may emit before it hands over: 4096 (config 4's closed forms fit), fewer for
// batches of more than 512 files so that the pinned event buffer stays within 64 MiB
constexpr int32_t kChainEventsMax = 4096;
constexpr int64_t kChainEventBytes = 64ll << 20;

inline int64_t pad16(int64_t v) { return (v + kPad - 1) / kPad * kPad; }

inline BatchState* state_of(rsh_ctx* c) {
    if (!c->batch) c->batch = new (std::nothrow) BatchState();
    return c->batch;
}

template <class T>
hipError_t pin(PinnedBuf& b, int64_t count, T** out) {
    const hipError_t e = b.ensure((size_t)std::max<int64_t>(count, 1) * sizeof(T));
    *out = b.as<T>();
    return e;
}

#define RSH_BHIP(call)                                  \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) {                         \
            note_error(e_, __LINE__, __FILE__);         \
            return RSH_E_DEVICE;                        \
        }                                               \
    } while (0)

// ------------------------------------------------------------------------------------------------
// Sender batch
// ------------------------------------------------------------------------------------------------
struct Req {
    // WAIT: until the speculation lands (no device work); FLUSH: WEAK at pos + BYTES at pos2 (one round trip);
    // FCHAIN: the batched flush chain in one round trip -- FLUSH's gathers into device memory, the chain on the
    // device (fchain; chain_out gets every step's desync), then PROBE over iv[0, niv), whose entries from npre on
    // are the chain's intervals with the desync the chain kernel writes
    enum Kind { WEAK, BYTES, WIN, PROBE, WAIT, FLUSH, FCHAIN } kind = WEAK;
    const int64_t* pos = nullptr;  // WEAK / BYTES / FLUSH (weak sums)
    int64_t count = 0;
    const int64_t* pos2 = nullptr;  // FLUSH: byte positions
    int64_t count2 = 0;
    uint8_t* out_b2 = nullptr;
    int32_t* out_w = nullptr;
    uint8_t* out_b = nullptr;
    int64_t p = 0, w = 0;          // WIN: window [p, p + w) lands at win
    const uint8_t* win = nullptr;
    const ProbeInterval* iv = nullptr;  // PROBE
    int64_t niv = 0;
    const std::vector<int32_t>* keys = nullptr;
    bool head = false;
    int64_t result = -1;
    const ProbeOut* out = nullptr;  // the probe's full answer (pinned), for the hit cache
    FlushChain fchain;              // FCHAIN
    int64_t npre = 0;
    uint32_t* chain_out = nullptr;  // FCHAIN: 2 K words
};

struct Batch;

class BatchBackend : public ScanBackend {
  public:
    Batch* b = nullptr;
    int32_t f = 0;
    bool head = true;
    int64_t na = 0;
    const int32_t* aw = nullptr;
    const uint8_t* as = nullptr;
    const uint8_t* fl = nullptr;
    const uint8_t* win0 = nullptr;  // window 0 (pinned), w0 bytes
    int64_t w0 = 0;
    const uint8_t* hit = nullptr;   // this file's hit buffer (pinned): T(p), then the window at p
    const int32_t* bucket = nullptr;
    int64_t n = 0, B = 0;
    uint8_t seed[4];
    ChunkTable* table = nullptr;
    std::vector<uint8_t> haw_ready;
    int64_t win_pos[HIT_WINDOWS] = {-1, -1, -1, -1};  // the last probe's hits whose windows are in `hit`
    int64_t t_pos = -1;    // the last hit returned: its weak sum t_val is known
    int32_t t_val = 0;
    HitCache cache;
    // read-ahead of window requests: the bytes [pf_pos, pf_pos + pf.size()) of the source, copied with the
    // last window request; a later digest inside them needs no round trip (in head mode the next match of
    // a chain, or of every other block, is usually a window or two further on)
    std::vector<uint8_t> pf;
    int64_t pf_pos = -1;

    int64_t aligned_count() override;
    int64_t flags_count() override { return head ? 0 : na; }
    int64_t max_batch() override { return head ? 4 : 4096; }
    const int32_t* aligned_weak() override { return aw; }
    const uint8_t* aligned_strong() override { return as; }
    const uint8_t* chain_flags() override { return fl; }
    void weak_many(const int64_t* pos, int64_t count, int32_t* out) override;
    void bytes_many(const int64_t* pos, int64_t count, uint8_t* out) override;
    void flush_gather(const int64_t* tpos, int64_t nt, int32_t* tv, const int64_t* bpos, int64_t nb,
                      uint8_t* bv) override;
    void md5_at(int64_t p, uint8_t out[16]) override;
    int64_t first_hit(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys) override;
    int64_t flush_probe(const ProbeInterval* pre, int64_t npre, const FlushChain& q, std::vector<FlushStep>* steps,
                        std::vector<ProbeInterval>* ivs, const std::vector<int32_t>* keys) override;
  private:
    int64_t probe_answer(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys);
};

struct FileScan {
    int32_t job = 0;
    const uint8_t* d_src = nullptr;
    const int32_t* d_weak = nullptr;
    const uint8_t* d_strong = nullptr;
    int64_t n = 0, B = 0, na = 0, nf = 0;
    int64_t na_a = 0;  // two-phase chain walk: the windows of its prefix speculation (na: one phase)
    int64_t lane_b_bytes = 0;  // bytes of its phase-1 lane chunks (they poll no abort word: they always run)
    const rsh_event* dev_ev = nullptr;  // a file the chain walk finished: its events, in the walk's pinned buffer
    int64_t dev_n = 0;
    int32_t C = 0, dl = 0;
    uint32_t ns = 0;
    int64_t off_tw = 0, off_ts = 0, off_na = 0, off_as = 0, off_nf = 0, off_ns = 0, off_hit = 0, off_w0 = 0;
    ChunkTable table;
    ResolveState rs;
    ResolveResult res;
    BatchBackend be;
    // rendezvous: the resolver runs as a fiber on one of the batch's worker threads
    Req req;
    bool pending = false;
    bool done = false;
    bool started = false;
    bool cancelled = false;  // its speculation groups were dropped or told to stop (file_abort)
    bool wait_spec = false;  // its lead windows carry their chunks' sums: wait for the speculation, no head mode
    int32_t worker = 0;
    ucontext_t uc;
    char* stack = nullptr;  // BatchState::fiber_stacks[i] for the i-th live file (reused across scans)
};

// Rounds: W worker threads (one per host core of the process, at most kMaxWorkers) each own a share of
// the resolvers, run as fibers (ucontext): a resolver that needs the device posts its request and switches
// back to its worker, which runs its next resolver.  When every worker has run all its resolvers up to
// their next request (or their end), the coordinator serves the round and starts the next one.  No more
// OS threads than cores, so a round's host work (digests of hit windows, bucket lookups) is not stretched
// by the scheduler.
struct Batch {
    std::mutex mu;
    std::condition_variable cv_coord, cv_work;
    // written under mu (the condition variables' predicates); atomic so that a waiter can spin on them
    // before it blocks (spin_wait)
    std::atomic<int32_t> idle{0};
    std::atomic<int32_t> nworkers{0};  // workers with a live file (a worker leaves once all of its files are done)
    std::atomic<uint64_t> gen{0};
    std::atomic<bool> quit{false};
    std::atomic<bool> landed{false};   // the speculation's chain flags are on the host (resolvers leave head mode)
    std::atomic<bool> aligned{false};  // ... and its aligned sums (aligned lookups)
    std::vector<FileScan>* files = nullptr;
    std::vector<ucontext_t> worker_uc;
    std::vector<double> busy_ms, max_fiber_ms;  // per worker, this round (trace)
    std::vector<HostTimes> times;               // per worker, cumulative (trace)

    // early resolution (match_scan_batch_claimed, while other walks still run): a request is served at once, on
    // the coordinator's thread, by this
    std::function<void(FileScan&)> direct;
    // in a resolver fiber: hand the request to the coordinator, yield to the worker until it is answered
    void post(FileScan& fs) {
        if (direct) {
            direct(fs);
            return;
        }
        fs.pending = true;
        swapcontext(&fs.uc, &worker_uc[(size_t)fs.worker]);
    }
};


inline FileScan& scan_of(Batch* b, int32_t f) { return (*b->files)[(size_t)f]; }

inline int64_t BatchBackend::aligned_count() { return (head || !b->aligned.load(std::memory_order_acquire)) ? 0 : na; }

// Round hand-offs: a blocked thread takes ~50 us to wake from a condition variable, once per round per
// side (coordinator -> workers, last worker -> coordinator).  Waiters spin up to RSH_BATCH_SPIN us
// (option batch_spin_us, default 200; 0 = block at once) on the predicate first, then block as before; the
// predicate is re-checked under the mutex either way, so the hand-off protocol is unchanged.
inline int spin_us() { return (int)std::max<int64_t>(0, opt(OPT_BATCH_SPIN_US)); }
template <class Pred>
void spin_wait(Pred pred) {
    const int us = spin_us();
    if (us <= 0 || pred()) return;
    const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(us);
    for (uint32_t i = 1;; ++i) {
        __builtin_ia32_pause();
        if (pred()) return;
        if ((i & 63) == 0) {
            if (std::chrono::steady_clock::now() >= end) return;
            sched_yield();
        }
    }
}

// batch_pool.cpp: a wait that polls an event, and one for everything enqueued on st so far (the rounds' latency path)
hipError_t spin_event(hipEvent_t ev);
hipError_t spin_sync(BatchState* S, hipStream_t st);
// batch_pool.cpp: one round -- every pending request of `pend` answered with one launch per kind and one
// synchronisation; a HIP error leaves every request answered with "nothing" (the resolvers finish on it)
hipError_t serve_round(rsh_ctx* c, BatchState* S, std::vector<FileScan>& files, const std::vector<int32_t>& pend,
                       hipStream_t st);

// What the resolver pool's coordinator needs from scan_batch: the deferred speculation launch (launched after
// defer_rounds rounds unless it already runs) and the state it shares with scan_batch.
struct RoundCtl {
    std::function<int()> launch_spec;
    bool* spec_launched = nullptr;
    int* spec_rc = nullptr;
    int defer_rounds = 0;
    bool k1_launched = false;  // the speculation's K1 runs: cancel resolved files' groups (file_abort)
    int gen = 0;               // ... with this generation
    bool trace = false;
    std::chrono::steady_clock::time_point t0;
};
// batch_pool.cpp: the resolvers of the files not done yet, as fibers on W worker threads, rounds served by the calling
// thread until every file is done; returns the first HIP error of the rounds (the resolvers still ran to the end) and
// the round count in *rounds.  The workers are detached when it returns; they touch nothing but *bp afterwards.
hipError_t run_resolvers(rsh_ctx* c, BatchState* S, const std::shared_ptr<Batch>& bp, std::vector<FileScan>& files,
                         hipStream_t st, RoundCtl& ctl, int* rounds);

}  // namespace batch
}  // namespace rsh
