// scan.cpp -- the single-file Sender scan on the device (Sender.sendMatchesAndData, Sender.java:1235-1327): the
// buffers and warm-up of a context (ctx_warm), the device-resident scan (scan_device: the aligned speculation, the
// sampled launch decision, the phase guess and the resolver over HipBackend) and the tiled scan (scan_tiled, BASELINE
// config 3), and the event hand-out (emit_events).  The C-ABI entry points that call them are in capi.cpp.
#include "scan_backend.h"

namespace rshi {
// Under scan_spec_queue the aligned speculation's sums come down on aux after the scan has moved on (or returned):
// a K1 that rewrites src_weak / src_strong on the context stream first waits for that download, when it is still
// running (a host-side query: no wait packet in the common case).
// The stamped launches' device counters and pinned stamps (scan_device under scan_spec_queue): slot 0 the prep
// launch, slot 1 the chain flags.  prep_dev: each slot's counters (rsh::Stamp: the launch counter and its group
// counters, 64 B each), then the prep's scratch sums; zero when allocated, and every stamped launch leaves them zero.
constexpr size_t kStampBytes = 64 * (1 + rsh::kStampGroups), kPrepScratchAt = 2 * kStampBytes;
hipError_t prep_ensure(rsh_ctx* c, int64_t nsamp) {
    const size_t need = kPrepScratchAt + (size_t)(2 * nsamp + 2) * 4;
    if (c->prep_dev.cap < need) {
        hipError_t e = c->prep_dev.ensure(std::max<size_t>(need, 4096));
        if (e == hipSuccess) e = hipMemset(c->prep_dev.p, 0, c->prep_dev.cap);
        if (e != hipSuccess) return e;
    }
    if (!c->h_stamps.p) {
        const hipError_t e = c->h_stamps.ensure(4096);
        if (e != hipSuccess) return e;
        memset(c->h_stamps.p, 0, c->h_stamps.cap);
    }
    return hipSuccess;
}
uint32_t* prep_counter(rsh_ctx* c, int slot) {
    return reinterpret_cast<uint32_t*>(c->prep_dev.as<uint8_t>() + kStampBytes * slot);
}
int* prep_stamp(rsh_ctx* c, int slot) { return reinterpret_cast<int*>(c->h_stamps.as<uint8_t>() + 64 * slot); }

// Spins until a stamped launch has written `gen` into its stamp.  A launch that fails never writes it: after 10 s
// the stream is synchronised, which reports the failure.
hipError_t wait_stamp(const int* stamp, int gen, hipStream_t s) {
    const volatile int* v = stamp;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (*v == gen) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return hipSuccess;
        }
        _mm_pause();
        if ((i & 0x3FF) == 0 && ms_since(t0) > 0.2) std::this_thread::yield();  // a K1 takes milliseconds
        if ((i & 0xFFFF) == 0 && ms_since(t0) > 10000.0) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            return *v == gen ? hipSuccess : hipErrorLaunchFailure;
        }
    }
}

hipError_t spec_buffers_free(rsh_ctx* c) {
    if (!c->spec_dl_pending) return hipSuccess;
    c->spec_dl_pending = false;
    const hipError_t q = hipEventQuery(c->ev_rs_tail);
    if (q == hipSuccess) return hipSuccess;
    if (q != hipErrorNotReady) return q;
    return hipStreamWaitEvent(c->stream, c->ev_rs_tail, 0);
}

// the segmented K1's descriptors: a wave per 64 windows of the prefix and phase speculations, up to 256 tails
size_t scan_seg_bytes(int64_t na) { return ((size_t)na / 64 + 4) * sizeof(rsh::K1Seg) + 256 * sizeof(rsh::K1Tail); }

// The single-file scan's per-window and per-chunk buffers for a source of na windows against a table of C chunks
// (scan_device; ctx_warm sizes them once for a config-5 file).
hipError_t scan_buffers_ensure(rsh_ctx* c, int64_t C, int64_t dl, int64_t na, bool download) {
    const int64_t nf = std::min<int64_t>(na, C);
    const uint32_t ns = pow2_at_least(2 * (uint64_t)C + 2);
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t x) {
        if (e == hipSuccess) e = x;
    };
    if (download) {
        ok(c->h_weak.ensure((size_t)C * 4 + 4));
        ok(c->h_strong.ensure((size_t)C * dl + 1));
    }
    ok(c->slots.ensure((size_t)ns * sizeof(unsigned long long)));
    ok(c->src_weak.ensure((size_t)na * 4));
    ok(c->src_strong.ensure((size_t)na * dl + 1));
    ok(c->flags.ensure((size_t)nf + 1));
    ok(c->h_aw.ensure((size_t)na * 4));
    ok(c->h_as.ensure((size_t)na * dl + 1));
    ok(c->h_fl.ensure((size_t)nf + 1));
    ok(c->haw.ensure((size_t)na * 4));
    for (int i = 0; i < 2; ++i) {
        ok(c->ph_weak[i].ensure((size_t)na * 4));
        ok(c->ph_strong[i].ensure((size_t)na * dl + 1));
        ok(c->h_pw[i].ensure((size_t)na * 4));
        ok(c->h_ps[i].ensure((size_t)na * dl + 1));
    }
    ok(c->segs.ensure(scan_seg_bytes(na)));
    ok(c->h_segs.ensure(scan_seg_bytes(na)));
    return e;
}

// rsh_ctx_create, after the streams (a JVM pays a context's first call once per context).  The
// runtime loads a file's code object at the first launch of any of its kernels -- 1.8 ms for device.hip's, 0.6 ms
// for device_scan.hip's on the first config-5 step of a fresh context (rocprofv3 HIP API trace, profiles/r5) -- and
// the first scan allocated ~25 pinned buffers at ~90 us each, some on its critical path.  Here: one empty launch
// per code object, and the single-file scan's buffers at a config-5 size (2^17 windows and chunks, dl 16, B 128 KiB):
// ~13 MiB of pinned host memory and ~16 MiB of HBM per context, which a larger file grows as before.
hipError_t ctx_warm(rsh_ctx* c) {
    constexpr int64_t kC = 1 << 17, kDl = 16, kB = 128 << 10;
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t x) {
        if (e == hipSuccess) e = x;
    };
    ok(rsh::launch_warm_k1(c->stream));
    ok(rsh::launch_warm_scan(c->stream));
    ok(rsh::launch_warm_chain(c->stream));
    ok(rsh::launch_warm_io(c->stream));
    ok(scan_buffers_ensure(c, kC, kDl, kC, true));
    ok(prep_ensure(c, kLeadWindows + rsh::opt(rsh::OPT_SCAN_SAMPLES) + 1));
    constexpr size_t kSmall = 64 << 10;  // PinnedBuf's least allocation
    for (PinnedBuf* b : {&c->h_lead, &c->h_prep, &c->h_pend, &c->h_keys, &c->h_iv, &c->h_tiles, &c->h_ptiles,
                         &c->h_psegs, &c->h_first, &c->h_bucket, &c->h_files, &c->h_pos, &c->h_out})
        ok(b->ensure(kSmall));
    ok(c->h_win0.ensure((size_t)kB + 16));
    ok(c->h_win.ensure((size_t)kB));
    ok(c->h_hit.ensure(16 + (size_t)kScanWindows * kB));
    ok(c->partials.ensure(kSmall));
    ok(c->bucket.ensure(rsh::HIT_BUCKET_INTS * sizeof(int32_t)));
    ok(c->first.ensure(kFirstSlots * sizeof(rsh::ProbeOut)));
    ok(c->dslots.ensure(kSmall));
    ok(c->fc_dev.ensure(kSmall));  // the batched flush chain's gathers (a stale digest's first round trip)
    for (PinnedBuf* b : {&c->h_fjobs, &c->h_fout}) ok(b->ensure(kSmall));
    ok(c->h_fgw.ensure(512 << 10));  // ... its gather list at 4096 intervals
    // the batched scan's state for a config-4 shard (option batch_warm files of 128 MiB, B 8192; dl 4 covers dl 3)
    ok(rsh::batch_warm(c, (int32_t)rsh::opt(rsh::OPT_BATCH_WARM), 128LL << 20, 8192, 4));
    // the runtime's copy and fill paths, on each of the context's streams: the first D2H copy of a process took
    // 6.8 ms (the single-file scan's table download, its first call in a fresh process: scan_trace, profiles/r5)
    if (e == hipSuccess) {
        uint8_t* d = c->slots.as<uint8_t>();
        uint8_t* hp = c->h_keys.as<uint8_t>();
        for (hipStream_t st : {c->stream, c->aux, c->phase}) {
            ok(hipMemsetAsync(d, 0, 4096, st));
            ok(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d + 4096), 0, 1024, st));
            ok(hipMemcpyAsync(hp, d, 4096, hipMemcpyDeviceToHost, st));
            ok(hipMemcpyAsync(d + 8192, hp, 4096, hipMemcpyHostToDevice, st));
            ok(hipMemcpyAsync(d + 12288, d, 4096, hipMemcpyDeviceToDevice, st));
            // a table-sized download (h_weak: C 4 + 4) the way the scan makes it (copy_to_host); the copy engine's
            // table-sized D2H is no longer on any scan path, and the profiler's async-copy tracing never saw its
            // completion (one per stream here: r5z2 copycb_files, hipMemcpyAsync of 512 KiB into pinned memory)
            ok(copy_to_host({rsh::CopyEnt{d, c->h_weak.as<uint8_t>(), 512 << 10}}, st));
            // the stream-write path (the runtime's own blit kernel): the abort of a stopped speculation
            ok(hipStreamWriteValue32(st, d + 16384, 0, 0));
            ok(hipStreamSynchronize(st));
        }
    }
    ok(hipStreamSynchronize(c->stream));
    // a host thread: every scan digests window 0 on one (glibc keeps the stack of a finished thread for the next)
    std::thread([] {}).join();
    return e;
}

// The device-resident Sender scan (everything but the whole-file MD5).  h validated by the caller;
// n > 0, block_length > 0.  host_weak/host_strong may be null (then copied back from the device).
//
// Streams (two per context, so that contexts rarely share one of the device's few hardware queues):
// `aux` downloads the received table and then runs the aligned speculation (K1 over the source +
// chain flags + their download); `stream` builds the probe hash and carries the resolver's small
// round trips.  The resolver starts in head mode as soon as the table is sorted, while the speculation
// is still running; when the speculation lands it resumes with it.  If the scan ends first -- e.g. the
// stale digest (quirk B) matches no chunk, after which only the closed-form flushes remain -- the
// speculation launch is told to stop (abort word) and its results are never read.
int scan_device(rsh_ctx* c, const uint8_t* d_src, int64_t n, const rsh_header* h, const int32_t* d_weak,
                const uint8_t* d_strong, const int32_t* host_weak, const uint8_t* host_strong, const uint8_t seed[4],
                rsh::ResolveResult* res) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t B = h->block_length;
    const int32_t C = h->chunk_count;
    const int32_t dl = h->digest_length;
    const int64_t na = (n + B - 1) / B;
    if (na > 2147483647LL) return RSH_E_OVERFLOW;
    const int64_t nf = std::min<int64_t>(na, C);
    const uint32_t ns = pow2_at_least(2 * (uint64_t)C + 2);

    // every buffer first (hipMalloc may synchronise), then the asynchronous work
    const bool download = !host_weak || !host_strong;
    RSH_HIP(scan_buffers_ensure(c, C, dl, na, download));
    const size_t seg_bytes = scan_seg_bytes(na);
    // sample windows for the launch decision: the first nlead, then one every `stride` windows
    const int64_t nlead = std::min<int64_t>(kLeadWindows, nf);
    const int64_t nsamples = std::max<int64_t>(1, rsh::opt(rsh::OPT_SCAN_SAMPLES));
    const int64_t stride = std::max<int64_t>(1, (nf + nsamples - 1) / nsamples);
    std::vector<int64_t> samp;
    for (int64_t k = 0; k < nlead; ++k) samp.push_back(k);
    const int64_t samp_j0 = std::max<int64_t>(1, (nlead + stride - 1) / stride);  // the first multiple kept
    for (int64_t k = samp_j0 * stride; k < nf; k += stride) samp.push_back(k);
    const int64_t nsamp = (int64_t)samp.size();
    const size_t lead_ents_at = ((size_t)(nsamp + 1) * 4 + 63) & ~(size_t)63;
    RSH_HIP(c->h_lead.ensure(lead_ents_at + (size_t)(nsamp + 1) * sizeof(rsh::GatherEnt) + sizeof(rsh::ScanFile)));

    // Queues (option scan_spec_queue, default 1).  1: the speculation runs on the context stream itself, queued
    // right behind whatever produced the inputs there (the Generator's K1 in the bench: no cross-queue hand-off
    // and no sample kernels between the two K1s), and the round trips -- window 0, the samples, the table, the
    // resolver -- on aux beside it.  0: round 4's layout, the speculation on aux after the sample kernels.
    const bool on_ctx = rsh::opt(rsh::OPT_SCAN_SPEC_QUEUE) != 0;
    hipStream_t ss = on_ctx ? c->stream : c->aux;  // the speculation
    hipStream_t rs = on_ctx ? c->aux : c->stream;  // the round trips
    if (on_ctx) RSH_HIP(prep_ensure(c, nsamp));     // the stamped launches' counters and stamps
    // (old layout) whatever produced the inputs on the caller's stream.  scan_spec_queue: no marker between the
    // producer and the speculation -- the prep launch's stamp (below) tells the host the inputs are complete, and
    // ev_in is recorded on aux once it has seen it.
    if (!on_ctx) RSH_HIP(hipEventRecord(c->ev_in, c->stream));
    // (aux) the aligned speculation: the source's own block sums with the basis header's B and dl,
    // the chain flags, and their download.  It is a bet on long runs of aligned matches; in head mode it
    // is launched only once the resolver has taken scan_defer_steps steps or scan_defer_us without finishing
    // (until then the resolver's round trips run on an otherwise idle device: a range probe beside the
    // speculation takes ~0.16 ms instead of tens of microseconds).
    int gen = c->next_gen();  // a stopped speculation's generation; a later launch takes a new one
    const int diag = (int)rsh::opt(rsh::OPT_SCAN_DIAG);  // diagnostics (options.h)
    int64_t spec_na = na;  // windows the speculation covers: all, or a prefix (sampled launch decision)
    // The speculation K1 starts after the sample kernels on the context stream (window 0's copy and the lead and
    // sample weak sums, ~50 us) rather than beside them: every K1 wave holds its SIMD for the whole launch, so
    // the waves that share their SIMDs with a VALU-heavy kernel set the launch's end (r2: 3.13 ms ordered
    // against 3.40-3.49 ms beside them; the step 6.48-6.58 against 6.67 ms).  Option scan_spec_order = 0 (A/B):
    // beside them.
    const bool spec_after_prep = rsh::opt(rsh::OPT_SCAN_SPEC_ORDER) != 0;
    bool prep_recorded = false;
    bool k1_timed = false;  // the speculation's K1 recorded ev_k1a / ev_k1b with its dispatch (no marker packets)
    int64_t spec_sums_na = -1;  // scan_spec_queue: windows of the launched speculation whose sums are still on the device
    int flags_gen = 0;          // > 0: the last launch's flags are stamped with this value (prep_stamp(c, 1))
    // the last launch's flags on the host: its stamp, or its ev_flags
    auto flags_landed = [&]() -> bool {
        if (flags_gen > 0) return *static_cast<volatile int*>(prep_stamp(c, 1)) == flags_gen;
        return hipEventQuery(c->ev_flags) != hipErrorNotReady;
    };
    auto wait_flags = [&]() -> hipError_t {
        return flags_gen > 0 ? wait_stamp(prep_stamp(c, 1), flags_gen, c->stream) : hipEventSynchronize(c->ev_flags);
    };
    auto launch_spec = [&]() -> int {
        const int64_t sn = std::min<int64_t>(n, spec_na * B);  // bytes: whole windows, or to the end
        const int64_t snf = std::min<int64_t>(spec_na, C);
        if (on_ctx) {
            RSH_HIP(spec_buffers_free(c));  // the previous scan's downloads of these buffers (aux) are done
            // (option time_spec) its own dispatch events: each costs the queue ~4.5 us after the kernel
            if (rsh::opt(rsh::OPT_TIME_SPEC) != 0) rsh::k1_timing_next(c->ev_k1a, c->ev_k1b);
        } else {
            RSH_HIP(hipStreamWaitEvent(c->aux, spec_after_prep && prep_recorded ? c->ev_prep : c->ev_in, 0));
            RSH_HIP(hipEventRecord(c->ev_k1a, c->aux));
        }
        const hipError_t e = rsh::launch_block_sums(d_src, sn, (uint32_t)B, (uint32_t)spec_na, (uint32_t)dl,
                                                    seed_word(seed), c->src_weak.as<int32_t>(),
                                                    c->src_strong.as<uint8_t>(), ss,
                                                    (diag & 2) ? nullptr : c->abort_word, gen);
        k1_timed = on_ctx && rsh::k1_timing_taken();
        if (on_ctx) rsh::k1_timing_next(nullptr, nullptr);
        RSH_HIP(e);
        if (!on_ctx) RSH_HIP(hipEventRecord(c->ev_k1b, c->aux));
        // the flags first (a run of matches needs nothing else), then the sums (aligned lookups off the run).  Under
        // scan_spec_queue the flags kernel writes them into pinned host memory itself (option scan_flags_host): a
        // D2H copy between two kernels on one queue left it idle 20-100 us (tools/queue_lat.hip case 8); round 2
        // measured no difference in the old layout (r2_ab2), where the copy was off the critical path.
        const bool flags_host = on_ctx && rsh::opt(rsh::OPT_SCAN_FLAGS_HOST) != 0;
        if (flags_host) {  // stamped: the host polls the stamp instead of waiting for an event
            flags_gen = c->next_stamp();
            RSH_HIP(rsh::launch_chain_flags_stamped(c->src_weak.as<int32_t>(), c->src_strong.as<uint8_t>(), d_weak,
                                                    d_strong, (uint32_t)snf, (uint32_t)dl, c->h_fl.as<uint8_t>(),
                                                    rsh::Stamp{prep_counter(c, 1), prep_stamp(c, 1), flags_gen}, ss));
        } else {
            flags_gen = 0;
            RSH_HIP(rsh::launch_chain_flags(c->src_weak.as<int32_t>(), c->src_strong.as<uint8_t>(), d_weak, d_strong,
                                            (uint32_t)snf, (uint32_t)dl, c->flags.as<uint8_t>(), ss));
            RSH_HIP(copy_to_host({rsh::CopyEnt{c->flags.as<uint8_t>(), c->h_fl.as<uint8_t>(), snf}}, ss));
        }
        RSH_HIP(hipEventRecord(c->ev_flags, ss));
        if (on_ctx) {
            // the sums come down on aux once the resolver first asks for them (HipBackend::aligned_count): on the
            // context stream they would hold up the caller's next launch (the next Generator K1), and an identical
            // file resolves from the flags alone
            spec_sums_na = spec_na;
            return RSH_OK;
        }
        RSH_HIP(copy_to_host({rsh::CopyEnt{c->src_weak.as<uint8_t>(), c->h_aw.as<uint8_t>(), spec_na * 4},
                              rsh::CopyEnt{c->src_strong.as<uint8_t>(), c->h_as.as<uint8_t>(), spec_na * dl}},
                             c->aux));
        RSH_HIP(hipEventRecord(c->ev_spec, c->aux));
        return RSH_OK;
    };
    const bool head = !(diag & 1);
    bool spec_launched = false;
    bool spec_tentative = false, tentative_stopped = false;
    if (!head || (diag & 4)) {  // scan_diag bit 2: launch at once even in head mode (A/B)
        const int rc = launch_spec();
        if (rc != RSH_OK) return rc;
        spec_launched = true;
    }
    // (stream + a host thread) the digest of window 0: the first event of a scan over a similar file is
    // at position 0, and its MD5 (one serial chain, ~0.13 ms for 128 KiB) then overlaps the first probe
    const int64_t w0 = std::min<int64_t>(B, n);
    RSH_HIP(c->h_win0.ensure((size_t)w0 + 16));
    int32_t* lead_w = c->h_lead.as<int32_t>();
    const int32_t* lead_tw = nullptr;  // scan_spec_queue: the table's weak sums at the sampled chunks (prep launch)
    if (on_ctx) {
        // (context stream) window 0, the lead and sample sums and the table's sums at those chunks in one stamped
        // launch right behind the inputs' producer, then (launch-then-confirm, below) the speculation right behind
        // it: the two K1s are apart by this launch only, and nothing runs beside the speculation's start (the sample
        // kernels on aux beside it cost it ~90 us, r5c/r5e traces)
        const size_t tw_at = 128;
        RSH_HIP(c->h_prep.ensure(tw_at + (size_t)(nsamp + 1) * 4 + 64));
        int32_t* tw = reinterpret_cast<int32_t*>(c->h_prep.as<uint8_t>() + tw_at);
        {  // the scan as a batch of one for later gathers (the prefix end's window sums)
            auto* ents = reinterpret_cast<rsh::GatherEnt*>(c->h_lead.as<uint8_t>() + lead_ents_at);
            auto* lf = reinterpret_cast<rsh::ScanFile*>(ents + nsamp + 1);
            *lf = rsh::ScanFile{};
            lf->data = d_src;
            lf->n = n;
            lf->B = (uint32_t)B;
        }
        const int prep_gen = c->next_stamp();
        rsh::ScanPrep P{};
        P.data = d_src;
        P.n = n;
        P.B = (uint32_t)B;
        P.nsamp = head ? (uint32_t)nsamp : 0u;
        const int64_t pieces_opt = rsh::opt(rsh::OPT_SCAN_PREP_PIECES);
        // 32 KiB per workgroup (4 for config 5's 128 KiB windows): 18 us per prep launch against 23 us at 16 KiB
        // (8 pieces: more workgroups to count done; r5n5 headline traces)
        P.pieces = (uint32_t)std::max<int64_t>(1, pieces_opt > 0 ? pieces_opt : std::min<int64_t>(8, (B + 32767) / 32768));
        P.nlead = (uint32_t)nlead;  // the kernel lists the samples itself (no host reads on its dependent chain)
        P.stride = stride;
        P.j0 = samp_j0;
        P.table_weak = d_weak;
        P.C = C;
        P.out_t = lead_w;
        P.out_w = tw;
        P.w0 = c->h_win0.as<uint8_t>();
        P.w0_len = w0;
        P.scratch = reinterpret_cast<int32_t*>(c->prep_dev.as<uint8_t>() + kPrepScratchAt);
        P.st = rsh::Stamp{prep_counter(c, 0), prep_stamp(c, 0), prep_gen};
        RSH_HIP(rsh::launch_scan_prep(P, ss));
        if (head && !spec_launched && nlead > 0 && rsh::opt(rsh::OPT_SCAN_EARLY) != 0 && na <= kRoundWindows &&
            (nlead >= kLeadWindows || nlead == nf)) {  // launch-then-confirm (below), right behind the prep launch
            const int rc = launch_spec();
            if (rc != RSH_OK) return rc;
            spec_launched = spec_tentative = true;
        }
        {
            CallTrace tr("prep_stamp", nsamp);
            RSH_HIP(wait_stamp(prep_stamp(c, 0), prep_gen, ss));
        }
        RSH_HIP(hipEventRecord(c->ev_in, rs));  // the inputs are complete (the host saw the stamp)
        lead_tw = tw;
    } else {
        RSH_HIP(rsh::launch_copy_to_host(d_src, w0, c->h_win0.as<uint8_t>(), rs));
    }
    // (stream) T(kB) of the first nlead aligned windows: when all of them carry chunk k's weak sum the
    // source very likely continues as an aligned run of matches (an unchanged or appended file), and the
    // speculation is launched at once instead of after a few head-mode steps
    if (!on_ctx && head && nlead > 0) {
        auto* ents = reinterpret_cast<rsh::GatherEnt*>(c->h_lead.as<uint8_t>() + lead_ents_at);
        auto* lf = reinterpret_cast<rsh::ScanFile*>(ents + nsamp + 1);
        *lf = rsh::ScanFile{};
        lf->data = d_src;
        lf->n = n;
        lf->B = (uint32_t)B;
        for (int64_t i = 0; i < nsamp; ++i) ents[i] = rsh::GatherEnt{samp[(size_t)i] * B, 0, 0};
        RSH_HIP(rsh::launch_window_weak(lf, ents, (uint32_t)nsamp, lead_w, rs));
    }
    if (!on_ctx && spec_after_prep) {
        RSH_HIP(hipEventRecord(c->ev_prep, rs));
        prep_recorded = true;
    }
    // (stream) the received table to the host (the lead check and the resolver), after the sample work: the
    // speculation waits for the samples only, and these copies and the hash build below run beside it.
    // (scan_spec_queue: after the lead check, which takes the table's sums at the samples from the prep launch,
    // so that a stopped tentative launch's abort does not queue behind these copies)
    auto table_work = [&]() -> int {
        if (download) {
            if (C > 0)
                RSH_HIP(copy_to_host(
                                     {rsh::CopyEnt{reinterpret_cast<const uint8_t*>(d_weak), c->h_weak.as<uint8_t>(),
                                                   (int64_t)C * 4},
                                      rsh::CopyEnt{d_strong, c->h_strong.as<uint8_t>(), (int64_t)C * dl}},
                                     rs));
            RSH_HIP(hipEventRecord(c->ev_tab, rs));
        }
        // (stream) the device probe hash
        RSH_HIP(rsh::launch_table_clear(c->slots.as<unsigned long long>(), ns, rs));
        RSH_HIP(rsh::launch_table_insert(c->slots.as<unsigned long long>(), ns - 1, d_weak, (uint32_t)C, rs));
        return RSH_OK;
    };
    auto table_wait = [&]() -> int {
        {
            CallTrace tr("table_dl", C);
            if (download) RSH_HIP(hipEventSynchronize(c->ev_tab));
        }
        // on the context's stream the host reads nothing this stream still writes (the prep launch's outputs came with
        // its stamp; the prefix end's gathers are waited for where they are read): the first probe is queued behind
        // the probe hash at once.  Otherwise the lead and sample sums (lead_w) and window 0 come down on this stream.
        if (!on_ctx) {
            CallTrace tr("hash_sync", ns);
            RSH_HIP(hipStreamSynchronize(rs));
        }
        return RSH_OK;
    };
    if (download) {
        host_weak = c->h_weak.as<int32_t>();
        host_strong = c->h_strong.as<uint8_t>();
    }
    if (!on_ctx) {
        const int rc = table_work();
        if (rc != RSH_OK) return rc;
    }

    // Launch-then-confirm: when one K1 round covers every window (na <= kRoundWindows), the speculation that
    // the lead decides on below is launched now, before the host knows the table, so it starts the moment the
    // Generator's work ends on the device; the lead check then keeps it or stops it (its waves leave after
    // their first two stages).  Larger sources wait for the samples (the launch may cover a prefix only).
    // (scan_spec_queue: launched above, right behind the prep launch.)
    const bool early_on = rsh::opt(rsh::OPT_SCAN_EARLY) != 0;  // A/B
    if (!on_ctx && head && !spec_launched && nlead > 0 && early_on && na <= kRoundWindows &&
        (nlead >= kLeadWindows || nlead == nf)) {
        const int rc = launch_spec();
        if (rc != RSH_OK) return rc;
        spec_launched = spec_tentative = true;
    }

    // (host) sort the table
    rsh::ChunkTable table;
    table.chunk_count = C;
    table.block_length = (int32_t)B;
    table.remainder = h->remainder;
    table.digest_length = dl;
    table.weak = host_weak;
    table.strong = host_strong;
    if (!on_ctx) {
        const int rc = table_wait();
        if (rc != RSH_OK) return rc;
    }
    // the digest of window 0 on a host thread, started once the lead check below has decided on the speculation: the
    // thread's creation (tens of microseconds) then no longer delays a tentative launch's stop
    uint8_t md5_0[16];
    std::thread md5_0_thread;
    auto start_md5_0 = [&] {
        md5_0_thread = std::thread([&] {
            rsh::HostMd5 hm;
            hm.update(c->h_win0.as<uint8_t>(), (size_t)w0);
            hm.update(seed, 4);
            hm.final(md5_0);
        });
    };
    if (!on_ctx) start_md5_0();
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{md5_0_thread};

    // the chain evidence of the first aligned windows (see above): launch the speculation now and let the
    // resolver wait for it rather than take head-mode steps beside it
    bool spec_wait = false;
    int64_t run_last = -1, run_miss = -1;  // a sampled run's last matching window, the first sample past it
    bool defer_prefix = false;             // the prefix speculation waits for the phase guess (below)
    // A/B switches (options.h; tests flip some of them)
    const bool guess_on = rsh::opt(rsh::OPT_SCAN_PHASE_GUESS) != 0;
    const bool seg_on = rsh::opt(rsh::OPT_SCAN_SEGMENTED) != 0;
    const bool wait_on = rsh::opt(rsh::OPT_SCAN_WAIT) != 0;
    const bool sample_on = rsh::opt(rsh::OPT_SCAN_SAMPLE) != 0;
    if (CallTrace::on()) fprintf(stderr, "[rsh] lead_check at %9.3f ms\n", ms_since(t0));
    if (head && nlead > 0 && (!spec_launched || spec_tentative)) {
        // the table's weak sum at sample i: from the prep launch (scan_spec_queue) or the downloaded table
        auto tw_at = [&](int64_t i) { return lead_tw ? lead_tw[i] : host_weak[samp[(size_t)i]]; };
        int64_t lead = 0;
        while (lead < nlead && lead_w[lead] == tw_at(lead)) ++lead;
        const bool eager = lead == nlead && (nlead >= kLeadWindows || nlead == nf);
        // The run may stop somewhere (an insert shifts everything after it to another phase, where the
        // phase-shifted speculation takes over): cover only up to the last sample that still matches, plus
        // one stride.  A K1 over a few waves is not free -- each lane digests its whole window serially, 1.9 ms
        // at B = 128 KiB -- but it lands well before a full launch (3.0-3.4 ms at 2 waves/SIMD), and the
        // phase-shifted launch that follows gets the whole chip.
        int64_t cover = na;
        if (eager && sample_on) {
            int64_t lastk = nlead - 1;
            for (int64_t i = nlead; i < nsamp; ++i)
                if (lead_w[i] == tw_at(i)) lastk = samp[(size_t)i];
            if (lastk + stride < nf) {
                cover = std::min<int64_t>(na, (lastk + stride + 64) & ~(int64_t)63);  // whole waves
                run_last = lastk;
                for (int64_t i = 0; i < nsamp && run_miss < 0; ++i)
                    if (samp[(size_t)i] > lastk) run_miss = samp[(size_t)i];
            }
        }
        if (spec_tentative && (!eager || cover < na)) {  // stop the tentative launch; later ones take a new generation
            CallTrace tr("spec_stop", cover);
            RSH_HIP(hipStreamWriteValue32(rs, c->abort_word, (uint32_t)gen, 0));
            gen = c->next_gen();
            spec_launched = spec_tentative = false;
            tentative_stopped = true;
            res->stats.speculation_aborted = 3;  // overwritten below if a later launch lands or is stopped
        }
        if (spec_tentative) {
            spec_wait = wait_on;
        } else if (eager) {
            spec_na = cover;
            if (cover < na && run_miss > 0 && guess_on && HipBackend::phase_on() && C >= 4) {
                defer_prefix = true;  // launched below, with the phase guess's speculation when there is one
            } else {
                const int rc = launch_spec();
                if (rc != RSH_OK) return rc;
                spec_launched = true;
            }
            spec_wait = wait_on;
        }
    }
    // The prefix end (below) needs the weak sums of the aligned windows between the run's last matching sample
    // and the first that does not: launched with the table's work (on_ctx: its hash sync then covers them) or, at
    // the latest, ahead of the guess's first probe, so that they land in a round trip the scan takes anyway
    const int64_t pe_lo = run_last + 1, pe_hi = std::min<int64_t>(run_miss, nf - 1), pe_cnt = pe_hi - pe_lo + 1;
    int32_t* pe_w = nullptr;
    int64_t pe_bytes = 0;
    hipError_t pe_err = hipSuccess;
    auto launch_pe = [&] {
        if (!(defer_prefix && guess_on && seg_on && run_miss > 0 && pe_cnt > 0 && pe_cnt <= 4096)) return;
        const size_t ents_at = ((size_t)pe_cnt * 4 + 63) & ~(size_t)63;
        pe_err = c->h_pend.ensure(ents_at + (size_t)pe_cnt * sizeof(rsh::GatherEnt));
        if (pe_err != hipSuccess) return;
        auto* pents = reinterpret_cast<rsh::GatherEnt*>(c->h_pend.as<uint8_t>() + ents_at);
        for (int64_t i = 0; i < pe_cnt; ++i) pents[i] = rsh::GatherEnt{(pe_lo + i) * B, 0, 0};
        auto* lf = reinterpret_cast<rsh::ScanFile*>(reinterpret_cast<rsh::GatherEnt*>(c->h_lead.as<uint8_t>() + lead_ents_at) +
                                                    nsamp + 1);
        pe_err = rsh::launch_window_weak(lf, pents, (uint32_t)pe_cnt, c->h_pend.as<int32_t>(), rs);
        if (pe_err != hipSuccess) return;
        pe_w = c->h_pend.as<int32_t>();
        pe_bytes = pe_cnt * B;
    };
    if (on_ctx) {  // (aux) the table and the probe hash, after a tentative launch's abort (above)
        int rc;
        {
            CallTrace tr("table_work", C);
            rc = table_work();
        }
        if (rc == RSH_OK) launch_pe();
        start_md5_0();  // beside the table's download
        if (rc == RSH_OK) {
            CallTrace tr("table_wait", C);
            rc = table_wait();
        }
        if (rc != RSH_OK) return rc;
    }
    if (CallTrace::on()) fprintf(stderr, "[rsh] resolver   starts at %9.3f ms\n", ms_since(t0));
    HipBackend be(c, d_src, n, table, d_weak, seed);
    be.rs_ = rs;
    be.table.slots = c->slots.as<unsigned long long>();
    be.table.mask = ns - 1;
    be.aw = c->h_aw.as<int32_t>();
    be.as = c->h_as.as<uint8_t>();
    be.fl = c->h_fl.as<uint8_t>();
    be.head = head;
    be.md5_0 = [&](uint8_t out[16]) {
        if (md5_0_thread.joinable()) md5_0_thread.join();
        memcpy(out, md5_0, 16);
    };
    be.haw_ready.assign((size_t)na, 0);
    // Phase guess.  When the samples show the aligned run stopping (only a prefix speculated), the source most
    // likely goes on at another phase after an insert or delete (Sender.java:1282-1287: the scan then matches
    // chunks at kB + delta).  Look for that phase now -- the first position in [mB, mB + 2B), m the first sample
    // past the run, whose window and the next three carry four consecutive chunks' weak sums -- and start the
    // phase-shifted speculation there instead of once the resolver has walked the prefix.  A wrong guess is
    // stopped when the resolver hints another phase.  RSH_SCAN_PHASE_GUESS=0 (A/B) turns it off.
    int64_t guess = -1;
    if (!pe_w) launch_pe();
    RSH_HIP(pe_err);
    be.bytes_read += pe_bytes;
    if (guess_on && run_miss > 0 && (spec_launched || defer_prefix) && HipBackend::phase_on() && C >= 4) {
        CallTrace tr("phase_guess", run_miss);
        int64_t a = run_miss * B;
        const int64_t b = std::min<int64_t>(run_miss * B + 2 * B, n - 4 * B + 1);  // the edit may sit in window m
        // each probe: one round trip that also brings T at p + B, p + 2 B, p + 3 B (HipBackend::guess); the first
        // over the tile or two at a (a small edit puts the new phase a few bytes past the sample), the rest after
        be.guess = true;
        for (int tries = 0; tries < 8 && a < b && be.err == hipSuccess; ++tries) {
            const int64_t b1 = std::min(b, a + rsh::PROBE_TILE);
            rsh::ProbeInterval iv{a, b1, a, 0, 0};
            int64_t p = be.first_hit(&iv, 1, nullptr);
            if (p < 0 && b1 < b) {
                iv = rsh::ProbeInterval{b1, b, b1, 0, 0};
                p = be.first_hit(&iv, 1, nullptr);
            }
            if (p < 0) break;
            int32_t w[4];
            w[0] = be.weak_at(p);  // (came back with the probe)
            if (!be.guess_sums(p, w + 1)) {  // (a hit the previous probe's list answered: no sums came with it)
                const int64_t pos[3] = {p + B, p + 2 * B, p + 3 * B};
                be.weak_many(pos, 3, w + 1);
            }
            bool run = false;
            for (int64_t j = 0; j + 3 < C && !run; ++j)
                run = host_weak[j] == w[0] && host_weak[j + 1] == w[1] && host_weak[j + 2] == w[2] &&
                      host_weak[j + 3] == w[3];
            if (run) {
                guess = p;
                break;
            }
            a = p + 1;
        }
        be.guess = false;
    }
    // The prefix and the phase-shifted speculation in one segmented K1 launch: as two launches they need one
    // wave more than the chip's wave slots (each has a partial last wave), and that wave starts only when
    // another finishes (config 5's shift case: the phase launch landed after 5.4 ms instead of 3.9).  The
    // prefix ends at the first aligned window past the run whose weak sum is not its chunk's (found with one
    // gather); the phase windows start at the first window of the guessed phase at or after it; the two
    // segments' leftover chunks share the per-lane tail waves.
    bool seg_launched = false;
    if (defer_prefix && guess >= 0 && seg_on && be.err == hipSuccess) {
        CallTrace tr("seg_launch", guess);
        const int64_t k_lo = run_last + 1, k_hi = std::min<int64_t>(run_miss, nf - 1);
        const int64_t cnt = k_hi - k_lo + 1;
        hipDeviceptr_t lo = nullptr;
        size_t asize = 0;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(d_src);
        if (cnt > 0 && cnt <= 4096 && B % 128 == 0 && (B >> 7) >= 4 && (B >> 7) <= 1024 &&
            hipMemGetAddressRange(&lo, &asize, reinterpret_cast<hipDeviceptr_t>(const_cast<uint8_t*>(d_src))) ==
                hipSuccess) {
            std::vector<int32_t> w((size_t)cnt);
            if (pe_w && k_lo == pe_lo && cnt == pe_cnt) {  // launched with the guess (above); landed with its probes
                RSH_HIP(hipStreamSynchronize(rs));
                memcpy(w.data(), pe_w, (size_t)cnt * 4);
            } else {
                std::vector<int64_t> pos((size_t)cnt);
                for (int64_t i = 0; i < cnt; ++i) pos[(size_t)i] = (k_lo + i) * B;
                be.weak_many(pos.data(), cnt, w.data());
            }
            int64_t P = run_miss;  // aligned windows [0, P): up to the first one whose weak sum is not its chunk's
            for (int64_t i = 0; i < cnt; ++i)
                if (w[(size_t)i] != host_weak[k_lo + i]) {
                    P = k_lo + i;
                    break;
                }
            const int64_t s0 = guess - ((guess - P * B) / B) * B;  // the first window at the guess's phase >= P B
            const int64_t Q = (n - s0 + B - 1) / B;
            const uintptr_t alo = reinterpret_cast<uintptr_t>(lo), ahi = alo + asize;
            const uint32_t a0 = (uint32_t)(addr % 128), a1 = (uint32_t)((addr + (uintptr_t)s0) % 128);
            if (P > 0 && Q >= 8 && addr - a0 >= alo && be.err == hipSuccess) {
                auto* sg = reinterpret_cast<rsh::K1Seg*>(c->h_segs.p);
                int64_t wp = P / 64;  // full prefix waves whose lines (64 B + 128 bytes from d_src - a0) stay in it
                while (wp > 0 && addr - a0 + (uintptr_t)(wp * 64 * B) + 128 > ahi) --wp;
                int64_t wq = ((n - s0) / B) / 64;  // full phase waves whose lines stay in the allocation
                while (wq > 0 && addr + (uintptr_t)s0 - a1 + (uintptr_t)(wq * 64 * B) + 128 > ahi) --wq;
                const int gph = c->next_gen();
                const int pset = 1 - c->ph_set;  // the phase part's buffer set (HipBackend::phase_hint)
                uint32_t nseg = 0;
                for (int64_t v = 0; v < wp; ++v)
                    sg[nseg++] = rsh::K1Seg{d_src - a0 + v * 64 * B, c->src_weak.as<int32_t>() + v * 64,
                                            c->src_strong.as<uint8_t>() + v * 64 * dl, c->abort_word, gen, a0};
                for (int64_t v = 0; v < wq; ++v)
                    sg[nseg++] = rsh::K1Seg{d_src + s0 - a1 + v * 64 * B, c->ph_weak[pset].as<int32_t>() + v * 64,
                                            c->ph_strong[pset].as<uint8_t>() + v * 64 * dl,
                                            c->abort_word + rsh_ctx::kPhaseWord, gph, a1};
                auto* tl = reinterpret_cast<rsh::K1Tail*>(sg + nseg);
                uint32_t ntail = 0;
                for (int64_t k = wp * 64; k < P; ++k)
                    tl[ntail++] = rsh::K1Tail{d_src, n, c->src_weak.as<int32_t>(), c->src_strong.as<uint8_t>(),
                                              (uint32_t)k};
                for (int64_t k = wq * 64; k < Q; ++k)
                    tl[ntail++] = rsh::K1Tail{d_src + s0, n - s0, c->ph_weak[pset].as<int32_t>(),
                                              c->ph_strong[pset].as<uint8_t>(),
                                              (uint32_t)k};
                // full-length tails first (gathered into coalesced waves), the short last window after them
                const uint32_t nfull = (uint32_t)(std::stable_partition(tl, tl + ntail, [&](const rsh::K1Tail& t) {
                                                      return (int64_t)(t.c + 1) * B <= t.n;
                                                  }) - tl);
                const size_t bytes = nseg * sizeof(rsh::K1Seg) + ntail * sizeof(rsh::K1Tail);
                if (ntail <= 256 && bytes <= seg_bytes) {
                    spec_na = P;
                    const int64_t snf = std::min<int64_t>(P, C);
                    // the descriptors by a copy kernel on the launch's own stream: a copy-engine upload cost the
                    // launch ~20 us more (the engine's completion, then the compute queue's wait on it)
                    RSH_HIP(copy_to_host({rsh::CopyEnt{c->h_segs.as<uint8_t>(), c->segs.as<uint8_t>(), (int64_t)bytes}},
                                         ss));
                    if (on_ctx) RSH_HIP(spec_buffers_free(c));
                    else RSH_HIP(hipStreamWaitEvent(ss, c->ev_in, 0));
                    RSH_HIP(hipStreamWaitEvent(ss, c->ev_phase[pset], 0));
                    RSH_HIP(hipEventRecord(c->ev_k1a, ss));
                    RSH_HIP(hipEventRecord(c->ev_pha[pset], ss));
                    RSH_HIP(rsh::launch_block_sums_segments(c->segs.as<rsh::K1Seg>(), nseg,
                                                            reinterpret_cast<const rsh::K1Tail*>(
                                                                c->segs.as<uint8_t>() + nseg * sizeof(rsh::K1Seg)),
                                                            ntail, nfull, (uint32_t)B, (uint32_t)dl, seed_word(seed),
                                                            ss));
                    RSH_HIP(hipEventRecord(c->ev_k1b, ss));
                    RSH_HIP(hipEventRecord(c->ev_phb[pset], ss));
                    RSH_HIP(rsh::launch_chain_flags(c->src_weak.as<int32_t>(), c->src_strong.as<uint8_t>(), d_weak,
                                                    d_strong, (uint32_t)snf, (uint32_t)dl, c->flags.as<uint8_t>(),
                                                    ss));
                    RSH_HIP(copy_to_host({rsh::CopyEnt{c->flags.as<uint8_t>(), c->h_fl.as<uint8_t>(), snf}}, ss));
                    RSH_HIP(hipEventRecord(c->ev_flags, ss));
                    RSH_HIP(copy_to_host({rsh::CopyEnt{c->src_weak.as<uint8_t>(), c->h_aw.as<uint8_t>(), P * 4},
                                          rsh::CopyEnt{c->src_strong.as<uint8_t>(), c->h_as.as<uint8_t>(), P * dl}},
                                         ss));
                    RSH_HIP(hipEventRecord(c->ev_spec, ss));
                    RSH_HIP(copy_to_host({rsh::CopyEnt{c->ph_weak[pset].as<uint8_t>(), c->h_pw[pset].as<uint8_t>(), Q * 4},
                                          rsh::CopyEnt{c->ph_strong[pset].as<uint8_t>(), c->h_ps[pset].as<uint8_t>(),
                                                       Q * dl}},
                                         ss));
                    RSH_HIP(hipEventRecord(c->ev_phase[pset], ss));
                    c->ph_set = pset;
                    k1_timed = true;     // (the event records around it)
                    spec_sums_na = -1;   // its sums come down with it (above), not on request
                    flags_gen = 0;       // ... and its flags land with ev_flags (a stopped launch's stamp says nothing)
                    be.phase_adopt(s0, Q, gph, pset);
                    res->stats.phase_guesses++;
                    spec_launched = seg_launched = true;
                    // The resolver's first question past the prefix chain: the first hit in [P B, P B + 9 B] (synced
                    // state, the whole table; resolver.cpp step 2: window P is past the speculated windows, so
                    // its own sum is not known and the probe starts there).  Asked now, beside the launch, its
                    // answer and the window at the hit are in the backend's hit cache when the speculation
                    // lands, instead of a round trip after it (0.17-0.19 ms on the shift case).  Unused (and
                    // harmless) when the resolver asks elsewhere.  Option scan_preprobe = 0 (A/B).
                    const bool preprobe = rsh::opt(rsh::OPT_SCAN_PREPROBE) != 0;
                    const int64_t last = n - (h->remainder > 0 ? h->remainder : B);
                    const int64_t pa = P * B, pstop = std::min(P * B + 9 * B, last);
                    if (preprobe && P * B + 10 * B <= n && pa <= pstop && be.err == hipSuccess) {
                        const rsh::ProbeInterval iv{pa, pstop + 1, pa, 0, 0};
                        (void)be.first_hit(&iv, 1, nullptr);
                    }
                }
            }
        }
    }
    if (defer_prefix && !seg_launched) {  // the prefix alone, and the guess's speculation (if any) beside it
        const int rc = launch_spec();
        if (rc != RSH_OK) return rc;
        spec_launched = true;
        if (guess >= 0) {
            const int64_t before = be.ph_launches;
            be.phase_hint(guess - ((guess - run_last * B) / B) * B);  // from the run's last sampled window on
            res->stats.phase_guesses += be.ph_launches - before;
        }
    } else if (!defer_prefix && guess >= 0) {
        const int64_t before = be.ph_launches;
        be.phase_hint(guess - ((guess - run_last * B) / B) * B);
        res->stats.phase_guesses += be.ph_launches - before;
    }
    be.na = spec_na;
    be.partial = spec_na < na;
    rsh::ResolveState rstate;
    bool landed = false;
    int spec_rc = RSH_OK;
    const auto t_head = std::chrono::steady_clock::now();
    const bool done = rsh::resolve_run(n, table, be, &rstate, res, [&] {
        if (be.err != hipSuccess || !be.head) return true;
        CallTrace tr("ev_query", res->stats.head_steps);
        if (!spec_launched) {
            const int64_t defer_steps = rsh::opt(rsh::OPT_SCAN_DEFER_STEPS);
            const double defer_ms = (double)rsh::opt(rsh::OPT_SCAN_DEFER_US) / 1e3;
            // chain evidence: the scan just matched consecutive chunks, so long aligned runs are likely and
            // the speculation pays; otherwise (e.g. a false weak hit that poisons the digest, after which
            // the scan ends in closed form) it waits a little longer
            const bool chain = !res->ev.empty() && res->ev.back().kind == RSH_EV_MATCH && res->ev.back().count >= 2;
            if ((chain && res->stats.head_steps >= kChainSteps) || res->stats.head_steps >= defer_steps ||
                ms_since(t_head) >= defer_ms) {
                spec_rc = launch_spec();
                spec_launched = true;
                if (spec_rc != RSH_OK) return true;
                spec_wait = wait_on && chain;  // a run of matches: the speculation will carry the scan
            }
            if (!spec_wait) {
                res->stats.head_steps++;
                return false;
            }
        }
        if (spec_wait) {  // head-mode steps beside the launch would only slow it down
            CallTrace tw("spec_wait", res->stats.head_steps);
            landed = wait_flags() == hipSuccess;
            return true;
        }
        landed = flags_landed();
        if (!landed) res->stats.head_steps++;
        return landed;
    });
    if (spec_rc != RSH_OK) return spec_rc;
    if (be.err != hipSuccess) return RSH_E_DEVICE;
    bool spec_read = false;  // the aligned speculation ran to completion (its bytes count as read)
    if (done && !spec_launched) {
        // the scan ended in head mode before the speculation was needed (3: a tentative launch was stopped)
        if (res->stats.speculation_aborted != 3) res->stats.speculation_aborted = 2;
        // the stopped launch's waves leave within two stages; later work on this context starts after them
        if (tentative_stopped) RSH_HIP(hipStreamWaitEvent(rs, on_ctx ? c->ev_flags : c->ev_spec, 0));
        res->stats.device_ms += ms_since(t0);
    } else if (done && !landed && !flags_landed()) {
        RSH_HIP(hipStreamWriteValue32(rs, c->abort_word, (uint32_t)gen, 0));  // the rest is dead work
        // Later work on this context starts only once the stopped launch has left the CUs: K1 fills every
        // wave slot of the chip exactly once (2 per SIMD at 16 GiB, B = 128 KiB), and a launch that finds
        // slots still held by the draining waves (or their LDS fragmented) runs a second round of waves.
        if (!on_ctx) RSH_HIP(hipStreamWaitEvent(c->stream, c->ev_spec, 0));  // (on_ctx: it runs on the context stream)
        res->stats.speculation_aborted = 1;
        res->stats.device_ms += ms_since(t0);
    } else {
        RSH_HIP(wait_flags());  // the sums follow on aux; aligned_count() polls ev_spec
        res->stats.device_ms += ms_since(t0);
        res->stats.speculation_aborted = 0;
        spec_read = true;
        if (!done) {
            be.head = false;
            if (on_ctx && spec_sums_na >= 0) be.lazy_na = spec_sums_na;
            if (be.partial) {  // the prefix's anchors from the speculation, the rest on demand
                RSH_HIP(hipMemcpyAsync(c->haw.p, c->src_weak.p, (size_t)spec_na * 4, hipMemcpyDeviceToDevice, rs));
                std::fill(be.haw_ready.begin(), be.haw_ready.begin() + spec_na, (uint8_t)1);
            }
            CallTrace tr("resolve_end", res->stats.events);
            rsh::resolve_run(n, table, be, &rstate, res, nullptr);
        }
    }
    be.phase_stop();
    if (be.err != hipSuccess) return RSH_E_DEVICE;
    if (on_ctx) {  // the next K1 over src_weak / src_strong on the context stream waits for what aux still does
        RSH_HIP(hipEventRecord(c->ev_rs_tail, rs));
        c->spec_dl_pending = true;
    }
    res->stats.table_ms += table.sort_ms;  // 0 when the scan never needed the sorted table
    res->stats.device_bytes += be.bytes_read + (spec_read ? std::min<int64_t>(n, spec_na * B) : 0);
    c->spec_timed = spec_read && (!on_ctx || k1_timed);
    if (c->spec_timed) {
        float k1ms = 0.f;
        if (hipEventElapsedTime(&k1ms, c->ev_k1a, c->ev_k1b) == hipSuccess) res->stats.spec_kernel_ms = k1ms;
    }
    res->stats.phase_launches += be.ph_launches;
    res->stats.phase_kernel_ms += be.phase_ms;
    if (CallTrace::on()) fprintf(stderr, "[rsh] scan_body  %10lld %9.3f ms\n", (long long)n, ms_since(t0));
    return RSH_OK;
}

// The Sender scan over a source that HBM holds a tile at a time (BASELINE config 3: files larger than the
// device, FileView's sliding window over the file, FileView.java:235-278).  The table is on the device
// (d_weak, d_strong) and on the host; `fill` copies source bytes [off, off + len) into HBM.  One resolver
// over the whole file; its backend pages tiles of tile_T bytes (+ a 16 B halo) as the scan advances and
// runs the aligned speculation tile by tile.  Identical events to scan_device.
int scan_tiled(rsh_ctx* c, const std::function<hipError_t(uint8_t*, int64_t, int64_t)>& fill, int64_t n,
               const rsh_header* h, const int32_t* d_weak, const uint8_t* d_strong, const int32_t* host_weak,
               const uint8_t* host_strong, const uint8_t seed[4], int64_t tile_bytes, rsh::ResolveResult* res) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t B = h->block_length;
    const int32_t C = h->chunk_count;
    const int32_t dl = h->digest_length;
    const int64_t na = (n + B - 1) / B;
    if (na > 2147483647LL) return RSH_E_OVERFLOW;
    const uint32_t ns = pow2_at_least(2 * (uint64_t)C + 2);
    const int64_t T = std::max<int64_t>(16 * B, tile_bytes / B * B), H = 16 * B;
    const int64_t nf = std::min<int64_t>(na, C);
    RSH_HIP(c->data.ensure((size_t)std::min(n, T + H)));
    RSH_HIP(c->slots.ensure((size_t)ns * sizeof(unsigned long long)));
    RSH_HIP(c->src_weak.ensure((size_t)na * 4));
    RSH_HIP(c->src_strong.ensure((size_t)na * dl + 1));
    RSH_HIP(c->flags.ensure((size_t)nf + 1));
    RSH_HIP(c->h_aw.ensure((size_t)na * 4));
    RSH_HIP(c->h_as.ensure((size_t)na * dl + 1));
    RSH_HIP(c->h_fl.ensure((size_t)nf + 1));
    RSH_HIP(c->haw.ensure((size_t)na * 4));
    for (int i = 0; i < 2; ++i) {
        RSH_HIP(c->ph_weak[i].ensure((size_t)na * 4));
        RSH_HIP(c->ph_strong[i].ensure((size_t)na * dl + 1));
        RSH_HIP(c->h_pw[i].ensure((size_t)na * 4));
        RSH_HIP(c->h_ps[i].ensure((size_t)na * dl + 1));
    }
    RSH_HIP(spec_buffers_free(c));  // its tiles' K1s rewrite src_weak / src_strong on the context stream
    RSH_HIP(hipEventRecord(c->ev_in, c->stream));
    RSH_HIP(rsh::launch_table_clear(c->slots.as<unsigned long long>(), ns, c->stream));
    RSH_HIP(rsh::launch_table_insert(c->slots.as<unsigned long long>(), ns - 1, d_weak, (uint32_t)C, c->stream));
    RSH_HIP(hipStreamSynchronize(c->stream));
    rsh::ChunkTable table;
    table.chunk_count = C;
    table.block_length = (int32_t)B;
    table.remainder = h->remainder;
    table.digest_length = dl;
    table.weak = host_weak;
    table.strong = host_strong;
    HipBackend be(c, c->data.as<uint8_t>(), n, table, d_weak, seed);
    be.table.slots = c->slots.as<unsigned long long>();
    be.table.mask = ns - 1;
    be.na = na;
    be.aw = c->h_aw.as<int32_t>();
    be.as = c->h_as.as<uint8_t>();
    be.fl = c->h_fl.as<uint8_t>();
    be.tiled = true;
    be.tile_T = T;
    be.tile_H = H;
    be.tile_buf = c->data.as<uint8_t>();
    be.fill = fill;
    be.d_table_strong = reinterpret_cast<const int32_t*>(d_strong);
    be.haw_ready.assign((size_t)na, 0);
    be.ensure(0);
    if (be.err != hipSuccess) return RSH_E_DEVICE;
    rsh::resolve_scan(n, table, be, res);
    be.phase_stop();
    if (be.err != hipSuccess) return RSH_E_DEVICE;
    res->stats.device_ms += ms_since(t0);
    res->stats.table_ms += table.sort_ms;
    res->stats.device_bytes += be.bytes_read;
    res->stats.phase_launches += be.ph_launches;
    res->stats.phase_kernel_ms += be.phase_ms;
    res->stats.head_steps = be.tiles_loaded;  // tiled scans have no head mode: the count of tile loads
    return RSH_OK;
}

int emit_events(rsh_ctx* c, rsh::ResolveResult& r, rsh_event* ev, int64_t cap, int64_t* n_ev) {
    *n_ev = (int64_t)r.ev.size();
    if ((int64_t)r.ev.size() > cap || (!ev && !r.ev.empty())) {
        c->last_ev.swap(r.ev);  // rsh_fetch_events hands them out without a rescan
        return RSH_E_NOSPACE;
    }
    c->last_ev.clear();
    if (!r.ev.empty()) memcpy(ev, r.ev.data(), r.ev.size() * sizeof(rsh_event));
    return RSH_OK;
}

}  // namespace rshi
