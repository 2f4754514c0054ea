// batch.cpp -- the batched (multi-file) entry points of include/rsync_hip.h.
//
// Generator side: every file of a segment in one K1 launch (Generator.java:558-614 calls
// sendItemizeAndChecksums :866-909 once per file; here the per-chunk work of all of them is one grid).
//
// Sender side (Sender.sendFiles :1098-1148 -> sendMatchesAndData :1235-1327 per file): one resolver per
// file, each on its own host thread, exactly the single-file resolver (resolver.cpp).  A resolver's
// device questions (a range probe, weak sums or bytes at a few positions, a digest window) are posted to
// the batch and the thread blocks; once every live resolver is blocked or finished, the coordinator (the
// calling thread) answers all of them with one launch per kind and one stream synchronisation -- one
// round trip per round for the whole segment instead of one per question per file.  The aligned
// speculation (the sources' own block sums) is one batched K1 launch, deferred like the single-file
// scan's and cancelled when every resolver finishes first.
//
// This file plans a segment's scan and drives its chain walks (scan_batch); the resolvers the walks leave run in the
// pool of batch_pool.cpp, whose fiber scheduler's invariants are at the top of batch.h.
#include "batch.h"

namespace rsh {

void destroy_batch_state(BatchState* b) { delete b; }
hipError_t clear_batch_abort_words(BatchState* b) {  // (and the hit map's words: they carry a generation too)
    if (!b) return hipSuccess;
    hipError_t e = b->file_abort ? hipMemset(b->file_abort, 0, (size_t)b->file_abort_cap * 4) : hipSuccess;
    if (e == hipSuccess && b->chain_map.p) e = hipMemset(b->chain_map.p, 0, b->chain_map.cap);
    return e;
}

namespace batch {
namespace {

int scan_batch(rsh_ctx* c, rsh_scan_job* jobs, const std::vector<int32_t>& which, const uint8_t seed[4],
               rsh_scan_stats* agg) {
    BatchState* S = state_of(c);
    if (!S) return RSH_E_NOMEM;
    const auto t0 = std::chrono::steady_clock::now();
    const int32_t NF = (int32_t)which.size();
    std::vector<FileScan> files((size_t)NF);
    int64_t tw = 0, ts = 0, tna = 0, tas = 0, tnf = 0, tns = 0, thit = 0, tw0 = 0, maxC = 0;
    for (int32_t f = 0; f < NF; ++f) {
        FileScan& fs = files[(size_t)f];
        const rsh_scan_job& j = jobs[which[(size_t)f]];
        fs.job = which[(size_t)f];
        fs.d_src = static_cast<const uint8_t*>(j.d_src);
        fs.d_weak = static_cast<const int32_t*>(j.d_weak);
        fs.d_strong = static_cast<const uint8_t*>(j.d_strong);
        fs.n = j.n;
        fs.B = j.h.block_length;
        fs.C = j.h.chunk_count;
        fs.dl = j.h.digest_length;
        fs.na = (fs.n + fs.B - 1) / fs.B;
        fs.nf = std::min<int64_t>(fs.na, fs.C);
        fs.ns = pow2_at_least(2 * (uint64_t)fs.C + 2);
        fs.off_tw = tw, tw += fs.C;
        fs.off_ts = ts, ts += (int64_t)fs.C * fs.dl;
        fs.off_na = tna, tna += fs.na;
        fs.off_as = tas, tas += fs.na * fs.dl;
        fs.off_nf = tnf, tnf += fs.nf;
        fs.off_ns = tns, tns += fs.ns;
        fs.off_hit = thit, thit += pad16(16 + fs.B);  // one window per file (ScanFile::nwin = 1)
        fs.off_w0 = tw0, tw0 += pad16(std::min<int64_t>(fs.B, fs.n));
        maxC = std::max<int64_t>(maxC, fs.C);
    }
    // buffers first (allocation may synchronise), then the asynchronous work
    RSH_BHIP(S->h_weak.ensure((size_t)tw * 4 + 4));
    RSH_BHIP(S->h_strong.ensure((size_t)ts + 1));
    RSH_BHIP(S->slots.ensure((size_t)tns * 8));
    RSH_BHIP(S->src_weak.ensure((size_t)tna * 4));
    RSH_BHIP(S->src_strong.ensure((size_t)tas + 1));
    RSH_BHIP(S->flags.ensure((size_t)tnf + 1));
    RSH_BHIP(S->haw.ensure((size_t)tna * 4));
    RSH_BHIP(S->h_aw.ensure((size_t)tna * 4));
    RSH_BHIP(S->h_as.ensure((size_t)tas + 1));
    RSH_BHIP(S->h_fl.ensure((size_t)tnf + 1));
    RSH_BHIP(S->h_files.ensure((size_t)NF * sizeof(ScanFile)));
    RSH_BHIP(S->h_hit.ensure((size_t)thit));
    RSH_BHIP(S->h_win0.ensure((size_t)tw0));
    RSH_BHIP(S->first.ensure((size_t)NF * sizeof(ProbeOut)));
    RSH_BHIP(S->h_first.ensure((size_t)NF * sizeof(ProbeOut)));
    RSH_BHIP(S->bucket.ensure((size_t)NF * HIT_BUCKET_INTS * 4));
    RSH_BHIP(S->h_bucket.ensure((size_t)NF * HIT_BUCKET_INTS * 4));
    RSH_BHIP(S->h_copies.ensure((size_t)2 * NF * sizeof(CopyEnt)));
    RSH_BHIP(S->h_ccopies.ensure((size_t)NF * sizeof(CopyEnt) + (size_t)3 * NF * sizeof(CopyEnt)));
    RSH_BHIP(S->h_tabents.ensure((size_t)NF * sizeof(TableEnt)));
    RSH_BHIP(S->h_flagents.ensure((size_t)NF * sizeof(FlagEnt)));
    RSH_BHIP(S->h_flagents_a.ensure((size_t)NF * sizeof(FlagEnt)));
    std::vector<K1File> k1;
    for (FileScan& fs : files)
        k1.push_back(K1File{fs.d_src, fs.n, (uint32_t)fs.B, (uint32_t)fs.dl, (uint32_t)fs.na,
                            S->src_weak.as<int32_t>() + fs.off_na, S->src_strong.as<uint8_t>() + fs.off_as});
    std::vector<K1Plan> plans;
    std::vector<K1Lane> lanes;
    int lane_align = 16;
    bool partial = tail_gather_on();
    uint32_t ngroups = plan_block_sums_files(k1.data(), NF, &plans, &lanes, &lane_align, &partial);
    RSH_BHIP(S->ensure_file_abort(NF));
    for (K1Plan& pl : plans) pl.abort = S->file_abort + pl.file;
    // The chain walk (option batch_chain, with the default speculation policy) runs after the speculation.  Two
    // phases (option batch_chain_prefix): the speculation over each file's first na_a windows -- a quarter round of
    // the chip's wave slots over the whole batch (256 windows per file for config 4's 128 files: its 50%-modified
    // walks all end inside 2 MiB; a full round, 1024, cost that step 0.3 ms of prefix K1 and the identical one
    // 0.065 ms less, round 5 r5z6/r5z7) -- and a walk over them; then the rest of the speculation for the
    // files whose walk reached the prefix's end (the others' groups stop at once: the walk wrote their abort words)
    // and a second walk.  A file that leaves the synced state early (an edit) costs its prefix, not its whole length.
    const bool chain_on = opt(OPT_BATCH_CHAIN) != 0 && opt(OPT_BATCH_SPEC) == -1;
    const int32_t kChainEvents = (int32_t)std::clamp<int64_t>(
        kChainEventBytes / ((int64_t)std::max<int32_t>(NF, 1) * (int64_t)sizeof(rsh_event)), 256, kChainEventsMax);
    bool two_phase = false;
    std::vector<K1Plan> plans_a, plans_b;
    std::vector<K1Lane> lanes_a, lanes_b;
    int align_a = 16, align_b = 16;
    bool partial_a = tail_gather_on(), partial_b = tail_gather_on();
    uint32_t ng_a = 0, ng_b = 0;
    for (FileScan& fs : files) fs.na_a = fs.na;
    if (const int64_t pre = opt(OPT_BATCH_CHAIN_PREFIX); chain_on && pre != 0) {
        const int64_t P = pre > 0 ? pre : 16 * std::max<int64_t>(1, kWaveSlots / std::max<int32_t>(NF, 1));
        for (FileScan& fs : files) {
            fs.na_a = std::min(fs.na, P);
            two_phase = two_phase || fs.na_a < fs.na;
        }
    }
    if (two_phase) {
        std::vector<K1File> ka, kb;
        std::vector<int32_t> b_file;
        for (int32_t f = 0; f < NF; ++f) {
            FileScan& fs = files[(size_t)f];
            ka.push_back(K1File{fs.d_src, std::min<int64_t>(fs.n, fs.na_a * fs.B), (uint32_t)fs.B, (uint32_t)fs.dl,
                                (uint32_t)fs.na_a, S->src_weak.as<int32_t>() + fs.off_na,
                                S->src_strong.as<uint8_t>() + fs.off_as});
            if (fs.na_a == fs.na) continue;
            kb.push_back(K1File{fs.d_src + fs.na_a * fs.B, fs.n - fs.na_a * fs.B, (uint32_t)fs.B, (uint32_t)fs.dl,
                                (uint32_t)(fs.na - fs.na_a), S->src_weak.as<int32_t>() + fs.off_na + fs.na_a,
                                S->src_strong.as<uint8_t>() + fs.off_as + fs.na_a * fs.dl});
            b_file.push_back(f);
        }
        ng_a = plan_block_sums_files(ka.data(), (int32_t)ka.size(), &plans_a, &lanes_a, &align_a, &partial_a);
        ng_b = plan_block_sums_files(kb.data(), (int32_t)kb.size(), &plans_b, &lanes_b, &align_b, &partial_b);
        for (K1Plan& pl : plans_a) pl.abort = nullptr;  // the launch's word
        for (K1Plan& pl : plans_b) pl.abort = S->file_abort + b_file[(size_t)pl.file];
        // phase 1's lane chunks have no abort word: they read their bytes even for a file whose walk ended in the
        // prefix (the device-bytes stat counts them)
        for (const K1Lane& ln : lanes_b) {
            const int64_t lo = (int64_t)ln.c_first * ln.B, hi = std::min<int64_t>(ln.n, lo + (int64_t)ln.nchunks * ln.B);
            files[(size_t)b_file[(size_t)ln.file]].lane_b_bytes += std::max<int64_t>(0, hi - lo);
        }
    }
    RSH_BHIP(S->k1_groups.ensure(((size_t)std::max(ngroups, ng_a + ng_b) + 1) * sizeof(K1Group)));
    RSH_BHIP(S->k1_plans.ensure((std::max(plans.size(), plans_a.size() + plans_b.size()) + 1) * sizeof(K1Plan)));
    RSH_BHIP(S->k1_lanes.ensure((std::max(lanes.size(), lanes_a.size() + lanes_b.size()) + 1) * sizeof(K1Lane)));

    // per-file host state
    ScanFile* F = S->h_files.as<ScanFile>();
    // shared with the worker threads, which are detached once every resolver is done (they then only wake,
    // see quit and return: joining them would keep the call waiting for their exit)
    auto bp = std::make_shared<Batch>();
    Batch& b = *bp;
    b.files = &files;
    for (int32_t f = 0; f < NF; ++f) {
        FileScan& fs = files[(size_t)f];
        const rsh_scan_job& j = jobs[fs.job];
        fs.table.chunk_count = fs.C;
        fs.table.block_length = (int32_t)fs.B;
        fs.table.remainder = j.h.remainder;
        fs.table.digest_length = fs.dl;
        fs.table.weak = S->h_weak.as<int32_t>() + fs.off_tw;
        fs.table.strong = S->h_strong.as<uint8_t>() + fs.off_ts;
        BatchBackend& be = fs.be;
        be.b = &b;
        be.f = f;
        be.na = fs.na;
        be.aw = S->h_aw.as<int32_t>() + fs.off_na;
        be.as = S->h_as.as<uint8_t>() + fs.off_as;
        be.fl = S->h_fl.as<uint8_t>() + fs.off_nf;
        be.win0 = S->h_win0.as<uint8_t>() + fs.off_w0;
        be.w0 = std::min<int64_t>(fs.B, fs.n);
        be.hit = S->h_hit.as<uint8_t>() + fs.off_hit;
        be.bucket = S->h_bucket.as<int32_t>() + (int64_t)f * HIT_BUCKET_INTS;
        be.n = fs.n;
        be.B = fs.B;
        memcpy(be.seed, seed, 4);
        be.table = &fs.table;
        be.haw_ready.assign((size_t)fs.na, 0);
        F[f] = ScanFile{};
        F[f].data = fs.d_src;
        F[f].n = fs.n;
        F[f].B = (uint32_t)fs.B;
        F[f].out = S->first.as<ProbeOut>() + f;
        F[f].table_weak = fs.d_weak;
        F[f].C = fs.C;
        F[f].bucket = S->bucket.as<int32_t>() + (int64_t)f * HIT_BUCKET_INTS;
        F[f].hit = S->h_hit.as<uint8_t>() + fs.off_hit;
        F[f].nwin = 1;
        F[f].aligned_weak = S->haw.as<int32_t>() + fs.off_na;
    }

    hipStream_t st = c->stream, aux = c->aux;
    RSH_BHIP(hipEventRecord(c->ev_in, st));  // whatever produced the inputs on the context stream
    // (stream) windows 0 (their digests start on the host while the rest runs)
    CopyEnt* wc = S->h_ccopies.as<CopyEnt>();
    int64_t max_w0 = 0;
    for (int32_t f = 0; f < NF; ++f) {
        FileScan& fs = files[(size_t)f];
        const int64_t w0 = std::min<int64_t>(fs.B, fs.n);
        wc[f] = CopyEnt{fs.d_src, S->h_win0.as<uint8_t>() + fs.off_w0, w0};
        max_w0 = std::max(max_w0, w0);
    }
    RSH_BHIP(launch_copy_many(wc, (uint32_t)NF, max_w0, st));
    // (stream) T(kB) of each file's first lead windows (the launch decision below, as in scan_device)
    std::vector<int64_t> lead_at((size_t)NF + 1, 0);
    for (int32_t f = 0; f < NF; ++f)
        lead_at[(size_t)f + 1] = lead_at[(size_t)f] + std::min<int64_t>(kLeadWindows, files[(size_t)f].nf);
    const int64_t nlead_all = lead_at[(size_t)NF];
    const size_t lead_ents_at = ((size_t)(nlead_all + 1) * 4 + 63) & ~(size_t)63;
    RSH_BHIP(S->h_lead.ensure(lead_ents_at + (size_t)(nlead_all + 1) * sizeof(GatherEnt)));
    int32_t* lead_w = S->h_lead.as<int32_t>();
    if (nlead_all > 0 && !chain_on) {  // (the chain walk has no lead check)
        auto* ents = reinterpret_cast<GatherEnt*>(S->h_lead.as<uint8_t>() + lead_ents_at);
        for (int32_t f = 0; f < NF; ++f)
            for (int64_t k = 0; k < lead_at[(size_t)f + 1] - lead_at[(size_t)f]; ++k)
                ents[lead_at[(size_t)f] + k] = GatherEnt{k * files[(size_t)f].B, f, 0};
        RSH_BHIP(launch_window_weak(F, ents, (uint32_t)nlead_all, lead_w, st));
    }
    // the speculation K1 waits for the lead sums only (a VALU-heavy kernel beside it slows the waves that share
    // its SIMDs, and the slowest wave ends the launch); the tables' download and the probe hashes follow it on
    // the context stream and run beside the speculation (option scan_spec_order = 0, A/B: all of it beside)
    const bool spec_after_prep = opt(OPT_SCAN_SPEC_ORDER) != 0;
    if (spec_after_prep) RSH_BHIP(hipEventRecord(c->ev_prep, st));
    // (stream) the received tables, to pinned host memory in one kernel
    CopyEnt* tc = S->h_copies.as<CopyEnt>();
    int64_t max_tab = 0;
    uint32_t ntc = 0;
    for (FileScan& fs : files) {
        if (fs.C == 0) continue;
        tc[ntc++] = CopyEnt{reinterpret_cast<const uint8_t*>(fs.d_weak), S->h_weak.as<uint8_t>() + 4 * fs.off_tw,
                            (int64_t)fs.C * 4};
        if (fs.dl > 0)
            tc[ntc++] = CopyEnt{fs.d_strong, S->h_strong.as<uint8_t>() + fs.off_ts, (int64_t)fs.C * fs.dl};
        max_tab = std::max<int64_t>(max_tab, (int64_t)fs.C * 4);
    }
    // with the speculation after the lead sums, the table work below runs beside its K1: background launches
    // (priority 0, a few hundred workgroups; the download is PCIe-bound anyway).  Option batch_prep_all = 1
    // (A/B): the speculation after all of it, full-width launches.
    const bool prep_all = opt(OPT_BATCH_PREP_ALL) != 0;
    const bool bg = spec_after_prep && !prep_all;
    // (chain walks: the host tables and the probe hashes serve the resolvers only -- built after the walks, for
    // the files they leave)
    if (!chain_on) RSH_BHIP(launch_copy_many(tc, ntc, max_tab, st, bg));  // stream order: after whatever produced them
    RSH_BHIP(hipEventRecord(c->ev_tab, st));
    // (stream) the probe hashes
    TableEnt* te = S->h_tabents.as<TableEnt>();
    if (!chain_on) {
        RSH_BHIP(launch_table_clear(S->slots.as<unsigned long long>(), (uint64_t)tns, st, bg));
        for (int32_t f = 0; f < NF; ++f) {
            FileScan& fs = files[(size_t)f];
            te[f] = TableEnt{S->slots.as<unsigned long long>() + fs.off_ns, fs.d_weak, fs.ns - 1, fs.C};
        }
        RSH_BHIP(launch_table_insert_many(te, (uint32_t)NF, (int32_t)maxC, st, bg));
    }
    // The chain walk: the speculation runs at once for every file, and one launch walks each file's Sender state
    // machine on the device from its start for as long as the state stays synced and unpoisoned and every digest
    // it needs is speculated (device.hip chain_advance_kernel; two phases: see above).  The resolvers start where
    // the walks stopped -- files whose walk reached the end need none -- instead of taking one device round trip
    // per event from the start.  Its chunk indexes go here.
    if (chain_on) {
        RSH_BHIP(S->kslots.ensure(kslots_bytes(tns, tw)));
        RSH_BHIP(S->h_kents.ensure((size_t)NF * sizeof(ChunkIndexEnt)));
        RSH_BHIP(S->h_chain.ensure((size_t)NF * sizeof(ChainFile)));
        RSH_BHIP(S->h_chain_out.ensure((size_t)NF * sizeof(ChainOut)));
        RSH_BHIP(S->h_chain_ev.ensure((size_t)NF * kChainEvents * sizeof(rsh_event)));  // (kChainEvents: see above)
        if (!S->ev_fk) RSH_BHIP(hipEventCreateWithFlags(&S->ev_fk, hipEventDisableTiming));
        // the chunk indexes must be ready when the prefix K1 ends (the phase-0 walks wait for both): the runtime's
        // fill, then the index with several CASes in flight per thread; beside the prefix K1 (which holds every
        // wave slot) both end with it in config 4 (r3s: fill 0.06 ms + index 0.20 ms inside the K1's 0.29 ms)
        // (one fill clears the slots and the duplicate bytes behind them)
        RSH_BHIP(hipMemsetAsync(S->kslots.p, 0, (size_t)tns * 8 + (size_t)tw, st));
        ChunkIndexEnt* ke = S->h_kents.as<ChunkIndexEnt>();
        for (int32_t f = 0; f < NF; ++f) {
            FileScan& fs = files[(size_t)f];
            ke[f] = ChunkIndexEnt{TableEnt{S->kslots.as<unsigned long long>() + fs.off_ns, fs.d_weak, fs.ns - 1, fs.C},
                                  kslots_dup(S, tns) + fs.off_tw};
        }
        RSH_BHIP(launch_chunk_index(ke, (uint32_t)NF, (int32_t)maxC, st, bg));
    }
    if (spec_after_prep && prep_all) RSH_BHIP(hipEventRecord(c->ev_prep, st));

    // the batched aligned speculation (deferred; see scan_device in capi.cpp)
    int gen = c->next_gen();  // a stopped tentative launch's generation; a later launch takes a new one
    CopyEnt* sc = S->h_ccopies.as<CopyEnt>() + NF;
    // K1 over the sources needs nothing but the sources; the chain flags need the received tables (ev_in)
    bool k1_launched = false;
    auto launch_spec_k1 = [&]() -> int {
        k1_launched = true;
        // files already resolved (all workers idle here) need no speculation: their groups are dropped
        size_t kept = 0;
        ngroups = 0;
        for (const K1Plan& pl : plans)
            if (!files[(size_t)pl.file].done) {
                plans[kept] = pl;
                plans[kept++].g0 = ngroups;
                ngroups += pl.ng;
            }
        plans.resize(kept);
        kept = 0;  // the tail lanes too (they have no abort word: they are short)
        for (const K1Lane& ln : lanes)
            if (!files[(size_t)ln.file].done) lanes[kept++] = ln;
        lanes.resize(kept);
        int32_t dropped = 0;
        for (FileScan& fs : files)
            if (fs.done) fs.cancelled = true, ++dropped;
        if (opt(OPT_SCAN_TRACE))
            fprintf(stderr, "[rsh-batch] speculation launched: %u groups, %d resolved files dropped\n", ngroups, dropped);
        if (!S->ev_scopy) RSH_BHIP(hipEventCreateWithFlags(&S->ev_scopy, hipEventDisableTiming));
        if (S->scopy_pending) RSH_BHIP(hipEventSynchronize(S->ev_scopy));  // the previous scan's upload is done
        S->scopy_pending = false;
        RSH_BHIP(S->h_sgroups.ensure((plans.size() + 1) * sizeof(K1Plan)));
        RSH_BHIP(S->h_slanes.ensure((lanes.size() + 1) * sizeof(K1Lane)));
        if (!plans.empty()) {  // pinned staging: the upload does not block the coordinator
            memcpy(S->h_sgroups.p, plans.data(), plans.size() * sizeof(K1Plan));
            RSH_BHIP(hipMemcpyAsync(S->k1_plans.p, S->h_sgroups.p, plans.size() * sizeof(K1Plan), hipMemcpyHostToDevice,
                                    aux));
            RSH_BHIP(launch_expand_groups(S->k1_plans.as<K1Plan>(), (uint32_t)plans.size(), ngroups,
                                          S->k1_groups.as<K1Group>(), aux));
        }
        if (!lanes.empty()) {
            memcpy(S->h_slanes.p, lanes.data(), lanes.size() * sizeof(K1Lane));
            RSH_BHIP(hipMemcpyAsync(S->k1_lanes.p, S->h_slanes.p, lanes.size() * sizeof(K1Lane), hipMemcpyHostToDevice,
                                    aux));
        }
        RSH_BHIP(hipEventRecord(S->ev_scopy, aux));
        S->scopy_pending = true;
        // the sources may come from work on the context stream (and the lead sums go first, see above)
        RSH_BHIP(hipStreamWaitEvent(aux, (spec_after_prep && !chain_on) ? c->ev_prep : c->ev_in, 0));
        RSH_BHIP(launch_block_sums_batch(S->k1_groups.as<K1Group>(), ngroups, S->k1_lanes.as<K1Lane>(),
                                         (uint32_t)lanes.size(), lane_align, seed_word(seed), aux, c->abort_word, gen,
                                         partial));
        return RSH_OK;
    };
    auto launch_spec = [&]() -> int {
        if (!k1_launched) {
            const int r = launch_spec_k1();
            if (r != RSH_OK) return r;
        }
        RSH_BHIP(hipStreamWaitEvent(aux, c->ev_in, 0));
        FlagEnt* fe = S->h_flagents.as<FlagEnt>();
        uint32_t max_nf = 0, nsc = 0;
        int64_t max_len = 0;
        int64_t max_fl = 0;
        for (int32_t f = 0; f < NF; ++f) {  // the flags first (the chains need nothing else) ...
            FileScan& fs = files[(size_t)f];
            // a file resolved before the launch has no speculation: no flags, no downloads
            const uint32_t nflag = fs.cancelled ? 0u : (uint32_t)fs.nf;
            fe[f] = FlagEnt{S->src_weak.as<int32_t>() + fs.off_na, S->src_strong.as<uint8_t>() + fs.off_as, fs.d_weak,
                            fs.d_strong, S->flags.as<uint8_t>() + fs.off_nf, nflag, (uint32_t)fs.dl};
            max_nf = std::max<uint32_t>(max_nf, nflag);
            if (fs.cancelled || fs.nf == 0) continue;
            sc[nsc++] = CopyEnt{S->flags.as<uint8_t>() + fs.off_nf, S->h_fl.as<uint8_t>() + fs.off_nf, fs.nf};
            max_fl = std::max<int64_t>(max_fl, fs.nf);
        }
        const uint32_t nfl = nsc;
        for (int32_t f = 0; f < NF; ++f) {  // ... then the sums (aligned lookups off the chains)
            FileScan& fs = files[(size_t)f];
            if (fs.cancelled) continue;
            sc[nsc++] = CopyEnt{S->src_weak.as<uint8_t>() + 4 * fs.off_na, S->h_aw.as<uint8_t>() + 4 * fs.off_na,
                                fs.na * 4};
            if (fs.dl > 0)
                sc[nsc++] = CopyEnt{S->src_strong.as<uint8_t>() + fs.off_as, S->h_as.as<uint8_t>() + fs.off_as,
                                    fs.na * fs.dl};
            max_len = std::max<int64_t>(max_len, fs.na * 4);
        }
        RSH_BHIP(launch_chain_flags_many(fe, (uint32_t)NF, max_nf, aux));
        if (chain_on) RSH_BHIP(hipEventRecord(S->ev_fk, aux));
        // (chain walks: the host copies follow the walks, for the files they leave to the resolvers only)
        if (!chain_on) RSH_BHIP(launch_copy_many(sc, nfl, max_fl, aux));
        RSH_BHIP(hipEventRecord(c->ev_flags, aux));
        if (!chain_on) RSH_BHIP(launch_copy_many(sc + nfl, nsc - nfl, max_len, aux));
        RSH_BHIP(hipEventRecord(c->ev_spec, aux));
        return RSH_OK;
    };

    // policy (A/B via option batch_spec; the default (-1), measured best on config 4, is head mode with the
    // launch after kDeferRounds rounds): -2 "early" = the speculation's K1 starts now, beside whatever the
    // device is still doing (e.g. the Generator), resolvers in head mode until it lands; -3 "wait" = as
    // early, but the resolvers start only once it has landed; N >= 0 = launch after N rounds
    const int64_t pol_v = opt(OPT_BATCH_SPEC);
    const bool pol = pol_v != -1;
    const bool wait_spec = pol_v == -3;
    const bool early_spec = pol_v == -2 || wait_spec;
    const int defer_rounds = (pol && !early_spec) ? (int)std::max<int64_t>(0, pol_v) : kDeferRounds;
    // launch-then-confirm (default policy): the speculation K1 is launched now, behind the Generator's work;
    // the lead check below keeps it for the files whose first windows carry their chunks' sums (they wait for
    // it instead of taking head-mode rounds) or stops it when no file qualifies
    const bool early_on = opt(OPT_SCAN_EARLY) != 0;  // A/B
    const bool tentative = !pol && early_on && nlead_all > 0 && !chain_on;
    if (early_spec || tentative) {
        const int r = launch_spec_k1();
        if (r != RSH_OK) return r;
    }
    // A file's walk record into its resolver's state (prefix_only: the rest of the speculation is not used)
    std::vector<char> early((size_t)NF, 0);
    auto take_walk = [&](int32_t f, bool prefix_only) {
        const ChainOut* co = S->h_chain_out.as<ChainOut>();
        const rsh_event* ce = S->h_chain_ev.as<rsh_event>();
        FileScan& fs = files[(size_t)f];
        const ChainOut& o = co[f];
        if (o.status == CHAIN_DONE) {  // its events stay where the walk wrote them (copied once, at the end)
            fs.dev_ev = ce + (int64_t)f * kChainEvents;
            fs.dev_n = o.n_ev;
        } else {
            fs.res.ev.assign(ce + (int64_t)f * kChainEvents, ce + (int64_t)f * kChainEvents + o.n_ev);
        }
        fs.res.literal = o.literal;
        fs.res.matched = o.matched;
        fs.res.stats.chain_matches += o.chain_matches;
        fs.res.stats.events += o.events;
        fs.res.stats.flushes += o.flushes;
        fs.rs.s = o.s;
        fs.rs.m = o.m;
        fs.rs.pref = o.pref;
        fs.rs.anchor = o.s;
        fs.rs.elo = o.elo;  // (0, 0) but after a flush the walk took (CHAIN_WHY_FLUSHED)
        fs.rs.ehi = o.ehi;
        fs.rs.clear_from = o.clear_to >= 0 ? o.s : -1;  // the walk searched up to the flush point
        fs.rs.clear_to = o.clear_to;
        // a walk that stopped inside the prefix leaves only the prefix speculated (its file's other groups
        // stopped): the resolver's aligned lookups end there
        fs.be.na = (o.aborted || prefix_only) ? fs.na_a : fs.na;
        if (o.md5c_valid) {  // poisoned at an unaligned hit: the resolver goes on with the stale digest
            fs.rs.md5c.assign(o.md5c, o.md5c + fs.dl);
            fs.rs.md5c_valid = true;
            fs.rs.dkeys_ready = false;
        }
        if (o.status == CHAIN_DONE) fs.rs.done = fs.done = true;
    };
    // Early resolution.  Phase 0's walks end file by file (ChainOut::fin).  A walk that took a flush-point flush
    // (CHAIN_WHY_FLUSHED: poisoned and desynced) leaves its file to a stale digest's probe over the rest -- the
    // batched flush chain's one round trip -- which needs nothing the other walks produce: that file is resolved at
    // once, on the phase stream beside the walks still running (its table, probe hash and prefix sums copied there
    // first), instead of after the last walk.  Its requests are served on the coordinator's thread (Batch::direct).
    hipError_t early_err = hipSuccess;
    auto early_resolve = [&](int32_t f) -> hipError_t {
        FileScan& fs = files[(size_t)f];
        take_walk(f, true);
        if (fs.done) return hipSuccess;
        const auto te0 = std::chrono::steady_clock::now();
        hipStream_t es = c->phase;
        hipError_t e = S->h_early.ensure(4096);
        if (e != hipSuccess) return e;
        CopyEnt* ec = S->h_early.as<CopyEnt>();
        TableEnt* et = reinterpret_cast<TableEnt*>(ec + 8);
        uint32_t ne = 0;
        const int64_t nal = fs.na_a, nfl = std::min(fs.nf, nal);
        ec[ne++] = CopyEnt{reinterpret_cast<const uint8_t*>(fs.d_weak), S->h_weak.as<uint8_t>() + 4 * fs.off_tw, (int64_t)fs.C * 4};
        if (fs.dl > 0) ec[ne++] = CopyEnt{fs.d_strong, S->h_strong.as<uint8_t>() + fs.off_ts, (int64_t)fs.C * fs.dl};
        if (nfl > 0) ec[ne++] = CopyEnt{S->flags.as<uint8_t>() + fs.off_nf, S->h_fl.as<uint8_t>() + fs.off_nf, nfl};
        ec[ne++] = CopyEnt{S->src_weak.as<uint8_t>() + 4 * fs.off_na, S->h_aw.as<uint8_t>() + 4 * fs.off_na, nal * 4};
        if (fs.dl > 0)
            ec[ne++] = CopyEnt{S->src_strong.as<uint8_t>() + fs.off_as, S->h_as.as<uint8_t>() + fs.off_as, nal * fs.dl};
        et[0] = TableEnt{S->slots.as<unsigned long long>() + fs.off_ns, fs.d_weak, fs.ns - 1, fs.C};
        if ((e = hipStreamWaitEvent(es, S->ev_fa, 0)) != hipSuccess) return e;  // the prefix's sums and flags
        if ((e = launch_copy_many(ec, ne, std::max<int64_t>((int64_t)fs.C * 4, nal * 4), es)) != hipSuccess) return e;
        if ((e = launch_table_clear(S->slots.as<unsigned long long>() + fs.off_ns, fs.ns, es)) != hipSuccess) return e;
        if ((e = launch_table_insert_many(et, 1, fs.C, es)) != hipSuccess) return e;
        if ((e = spin_sync(S, es)) != hipSuccess) return e;
        fs.be.head = false;
        b.landed.store(true);
        b.aligned.store(true);
        const int32_t fi = f;
        b.direct = [&, fi](FileScan&) {
            const hipError_t x = serve_round(c, S, files, std::vector<int32_t>{fi}, es);
            if (x != hipSuccess && early_err == hipSuccess) early_err = x;
        };
        // (no eager sort: a stale digest's flush chain needs no bucket lookups; the index is built if a lookup comes)
        resolve_run(fs.n, fs.table, fs.be, &fs.rs, &fs.res, nullptr);
        b.direct = nullptr;
        fs.rs.done = fs.done = true;
        early[(size_t)f] = 1;
        if (opt(OPT_SCAN_TRACE))
            fprintf(stderr, "[rsh-batch] file %d resolved while the walks ran: %.3f ms, done at %.3f ms\n", f,
                    ms_since(te0), ms_since(t0));
        return early_err;
    };
    // the host's wait for phase 0's walks, taking up the files they hand over a flush-chain state early
    auto await_walks = [&]() -> hipError_t {
        const ChainOut* co = S->h_chain_out.as<ChainOut>();
        std::vector<char> seen((size_t)NF, 0);
        for (;;) {
            const hipError_t q = hipEventQuery(S->ev_wa);
            if (q != hipSuccess && q != hipErrorNotReady) return q;
            if (q == hipSuccess) return hipSuccess;  // the rest goes the usual way
            for (int32_t f = 0; f < NF; ++f) {
                if (seen[(size_t)f] || *reinterpret_cast<const volatile int32_t*>(&co[f].fin) == 0) continue;
                seen[(size_t)f] = 1;
                std::atomic_thread_fence(std::memory_order_acquire);
                if (co[f].status == CHAIN_STOP && co[f].why == CHAIN_WHY_FLUSHED) {
                    const hipError_t e = early_resolve(f);
                    if (e != hipSuccess) return e;
                }
            }
            _mm_pause();
        }
    };
    bool spec_launched = false;
    bool skip_rest = false;  // two phases, and phase 0 finished or handed over every file: no rest speculated
    if (chain_on) {  // the speculation, then the walks on the context stream (beside the sums' download on aux)
        ChainFile* cf = S->h_chain.as<ChainFile>();
        ChainOut* co = S->h_chain_out.as<ChainOut>();
        rsh_event* ce = S->h_chain_ev.as<rsh_event>();
        // the phase-0 hit map: each file whose walk may search tile by tile (wide tiles: B a multiple of 32, >= 512)
        // gets words for the positions [0, hend) its phase-0 searches may reach, if they all fit the budget
        std::vector<int64_t> map_off((size_t)NF + 1, 0);
        const int64_t helpers_opt = opt(OPT_CHAIN_HELPERS);
        bool map_on = two_phase && helpers_opt != 0;
        for (int32_t f = 0; map_on && f < NF; ++f) {
            const FileScan& fs = files[(size_t)f];
            const bool wide = fs.B >= 512 && fs.B % 32 == 0 && CHAIN_TILE / fs.B + 2 <= CHAIN_SEGS;
            const int64_t hend = std::min<int64_t>(fs.na_a * fs.B, fs.n - fs.B + 1);
            map_off[(size_t)f + 1] = map_off[(size_t)f] + (wide && fs.C > 0 && hend > 0 ? (hend + 31) / 32 : 0);
        }
        map_on = map_on && map_off[(size_t)NF] > 0 && map_off[(size_t)NF] * 8 <= opt(OPT_CHAIN_MAP_BYTES);
        if (map_on) {
            const size_t words = (size_t)map_off[(size_t)NF];
            if (words * 8 > S->chain_map.cap) {
                RSH_BHIP(S->chain_map.ensure(words * 8));
                RSH_BHIP(hipMemsetAsync(S->chain_map.p, 0, S->chain_map.cap, st));  // no stale generation
            }
            RSH_BHIP(S->chain_help.ensure((size_t)NF * sizeof(ChainHelp)));
            RSH_BHIP(S->h_chain_help.ensure((size_t)NF * sizeof(ChainHelp)));
        }
        ChainHelp* chh = map_on ? S->h_chain_help.as<ChainHelp>() : nullptr;
        for (int32_t f = 0; f < NF; ++f) {
            FileScan& fs = files[(size_t)f];
            co[f] = ChainOut{};
            co[f].clear_to = -1;
            const int64_t mw = map_on ? map_off[(size_t)f + 1] - map_off[(size_t)f] : 0;
            const int64_t hend = mw > 0 ? std::min<int64_t>(fs.na_a * fs.B, fs.n - fs.B + 1) : 0;
            cf[f] = ChainFile{fs.d_src, fs.n, (uint32_t)fs.B, fs.C, fs.dl, jobs[fs.job].h.remainder,
                              fs.ns - 1, S->kslots.as<unsigned long long>() + fs.off_ns, fs.d_weak, fs.d_strong,
                              S->src_weak.as<int32_t>() + fs.off_na, S->src_strong.as<uint8_t>() + fs.off_as,
                              S->flags.as<uint8_t>() + fs.off_nf, fs.na, fs.na_a,
                              two_phase ? S->file_abort + f : nullptr, ce + (int64_t)f * kChainEvents, kChainEvents,
                              seed_word(seed), co + f,
                              mw > 0 ? S->chain_map.as<unsigned long long>() + map_off[(size_t)f] : nullptr, hend,
                              kslots_dup(S, tns) + fs.off_tw};
            if (chh) chh[f] = ChainHelp{(int32_t)((hend + CHAIN_MAP_SEG - 1) / CHAIN_MAP_SEG), 0, 1, 0, 0, 0, 0, 0, INT64_MAX, 0, 0, 0,
                                        (int32_t)opt(OPT_CHAIN_HELP_TILES)};
        }
        const uint32_t n_help = !map_on ? 0u
                                : helpers_opt > 0 ? (uint32_t)helpers_opt
                                                  : (uint32_t)std::max<int64_t>(0, (int64_t)c->n_cu - NF);
        const bool tr = opt(OPT_SCAN_TRACE) != 0;
        if (tr) {  // the walks' own duration (trace only)
            for (hipEvent_t* e : {&S->ev_ch0, &S->ev_ch1})
                if (!*e) RSH_BHIP(hipEventCreate(e));
        }
        if (two_phase) {
            // phase 0: the prefix speculation (groups and lanes of both phases staged in one upload), its flags, the
            // walks over it; phase 1's K1 follows the walks, which stop the groups of the files they finished
            if (!S->ev_fa) RSH_BHIP(hipEventCreateWithFlags(&S->ev_fa, hipEventDisableTiming));
            if (!S->ev_wa) RSH_BHIP(hipEventCreate(&S->ev_wa));  // timed: the trace reports phase 0's walk
            if (!S->ev_scopy) RSH_BHIP(hipEventCreateWithFlags(&S->ev_scopy, hipEventDisableTiming));
            if (S->scopy_pending) RSH_BHIP(hipEventSynchronize(S->ev_scopy));  // the previous scan's upload is done
            S->scopy_pending = false;
            const size_t npa = plans_a.size(), npb = plans_b.size(), nla = lanes_a.size(), nlb = lanes_b.size();
            RSH_BHIP(S->h_sgroups.ensure((npa + npb + 1) * sizeof(K1Plan)));
            RSH_BHIP(S->h_slanes.ensure((nla + nlb + 1) * sizeof(K1Lane)));
            K1Plan* hp = S->h_sgroups.as<K1Plan>();
            std::copy(plans_a.begin(), plans_a.end(), hp);
            std::copy(plans_b.begin(), plans_b.end(), hp + npa);
            K1Lane* hl = S->h_slanes.as<K1Lane>();
            std::copy(lanes_a.begin(), lanes_a.end(), hl);
            std::copy(lanes_b.begin(), lanes_b.end(), hl + nla);
            if (npa + npb > 0)
                RSH_BHIP(hipMemcpyAsync(S->k1_plans.p, hp, (npa + npb) * sizeof(K1Plan), hipMemcpyHostToDevice, aux));
            if (npa > 0)
                RSH_BHIP(launch_expand_groups(S->k1_plans.as<K1Plan>(), (uint32_t)npa, ng_a, S->k1_groups.as<K1Group>(), aux));
            if (npb > 0)
                RSH_BHIP(launch_expand_groups(S->k1_plans.as<K1Plan>() + npa, (uint32_t)npb, ng_b,
                                              S->k1_groups.as<K1Group>() + ng_a, aux));
            if (nla + nlb > 0)
                RSH_BHIP(hipMemcpyAsync(S->k1_lanes.p, hl, (nla + nlb) * sizeof(K1Lane), hipMemcpyHostToDevice, aux));
            RSH_BHIP(hipEventRecord(S->ev_scopy, aux));
            S->scopy_pending = true;
            RSH_BHIP(hipStreamWaitEvent(aux, c->ev_in, 0));  // the sources only (no lead check in chain mode)
            RSH_BHIP(launch_block_sums_batch(S->k1_groups.as<K1Group>(), ng_a, S->k1_lanes.as<K1Lane>(), (uint32_t)nla,
                                             align_a, seed_word(seed), aux, c->abort_word, gen, partial_a));
            RSH_BHIP(hipStreamWaitEvent(aux, c->ev_in, 0));  // the flags need the received tables
            FlagEnt* fa = S->h_flagents_a.as<FlagEnt>();
            uint32_t max_na = 0;
            for (int32_t f = 0; f < NF; ++f) {
                FileScan& fs = files[(size_t)f];
                const uint32_t nflag = (uint32_t)std::min(fs.na_a, fs.nf);
                fa[f] = FlagEnt{S->src_weak.as<int32_t>() + fs.off_na, S->src_strong.as<uint8_t>() + fs.off_as, fs.d_weak,
                                fs.d_strong, S->flags.as<uint8_t>() + fs.off_nf, nflag, (uint32_t)fs.dl};
                max_na = std::max(max_na, nflag);
            }
            RSH_BHIP(launch_chain_flags_many(fa, (uint32_t)NF, max_na, aux));
            RSH_BHIP(hipEventRecord(S->ev_fa, aux));
            // the helpers' shared state goes up while the prefix K1 runs (behind the chunk indexes), not between the
            // flags and the walks
            if (map_on)
                RSH_BHIP(hipMemcpyAsync(S->chain_help.p, chh, (size_t)NF * sizeof(ChainHelp), hipMemcpyHostToDevice, st));
            RSH_BHIP(hipStreamWaitEvent(st, S->ev_fa, 0));
            const int gen_b = c->next_gen();
            if (tr) RSH_BHIP(hipEventRecord(S->ev_ch0, st));
            RSH_BHIP(launch_chain_advance(cf, (uint32_t)NF, st, 0, gen_b, map_on ? S->chain_help.as<ChainHelp>() : nullptr,
                                          n_help, tr));
            RSH_BHIP(hipEventRecord(S->ev_wa, st));
            // (option batch_skip_rest) once phase 0 has ended, the rest of the speculation only if some walk reached
            // the prefix's end (CHAIN_MORE): otherwise every file is done, or left to its resolver with the prefix
            // speculated, and the rest's launch -- all its groups stopping at once, ~0.17 ms of dispatch for config 4's
            // 30720 -- its flags and phase 1 are skipped.  The host waits for phase 0 either way (a few us more before
            // the rest's launch when it is needed).
            if (opt(OPT_BATCH_SKIP_REST) != 0 && opt(OPT_BATCH_CHAIN_OVERLAP) == 0) {
                RSH_BHIP(await_walks());
                skip_rest = true;
                for (int32_t f = 0; f < NF && skip_rest; ++f) skip_rest = co[f].status != CHAIN_MORE;
            }
            if (!skip_rest) {
                // the rest of the speculation after the walks (the groups of files they finished stop at once), or
                // (option batch_chain_overlap) beside them: no gap after the prefix's K1, but the walks share the chip
                if (opt(OPT_BATCH_CHAIN_OVERLAP) == 0) RSH_BHIP(hipStreamWaitEvent(aux, S->ev_wa, 0));
                RSH_BHIP(launch_block_sums_batch(S->k1_groups.as<K1Group>() + ng_a, ng_b, S->k1_lanes.as<K1Lane>() + nla,
                                                 (uint32_t)nlb, align_b, seed_word(seed), aux, c->abort_word, gen_b,
                                                 partial_b));
                k1_launched = true;
            }
            if (opt(OPT_SCAN_TRACE))
                fprintf(stderr, "[rsh-batch] two-phase speculation: prefix %u groups, rest %u groups%s\n", ng_a, ng_b,
                        skip_rest ? " (skipped: no walk reached the prefix's end)" : "");
        }
        if (!skip_rest) {
            const int r = launch_spec();  // (two phases: the flags of whole files and the downloads)
            if (r != RSH_OK) return r;
            spec_launched = true;
            RSH_BHIP(hipStreamWaitEvent(st, S->ev_fk, 0));
            if (tr && !two_phase) RSH_BHIP(hipEventRecord(S->ev_ch0, st));
            RSH_BHIP(launch_chain_advance(cf, (uint32_t)NF, st, two_phase ? 1 : 0, 0, nullptr, 0, tr));
        } else {  // what waits on the speculation's events below finds them complete (phase 0 is)
            RSH_BHIP(hipEventRecord(c->ev_flags, st));
            RSH_BHIP(hipEventRecord(c->ev_spec, st));
            RSH_BHIP(hipEventRecord(S->ev_fk, st));
            spec_launched = true;
        }
        if (tr) RSH_BHIP(hipEventRecord(S->ev_ch1, st));
    }
    const double enq_ms = ms_since(t0);
    RSH_BHIP(hipEventSynchronize(c->ev_tab));
    RSH_BHIP(spin_sync(S, st));
    const double setup_ms = ms_since(t0);

    const bool trace = opt(OPT_SCAN_TRACE) != 0;
    int spec_rc = RSH_OK;
    int32_t nwait = 0;
    if (chain_on) {  // the walks have ended (the stream sync above): each resolver resumes where its walk stopped
        const ChainOut* co = S->h_chain_out.as<ChainOut>();
        int32_t left = 0;
        for (int32_t f = 0; f < NF; ++f) {
            if (early[(size_t)f]) continue;  // resolved while the other walks ran
            take_walk(f, skip_rest);
            if (!files[(size_t)f].done) ++left;
        }
        b.landed.store(true);  // the walks ran after the speculation's K1 and flags
        if (left > 0) {  // the host resolvers use the speculation's host copies: the left files' flags and sums
            // the left files' received tables (host) and probe hashes (device) first
            uint32_t nt = 0, ntl = 0;
            int64_t mt = 0;
            for (FileScan& fs : files) {
                if (fs.done || fs.C == 0) continue;
                tc[nt++] = CopyEnt{reinterpret_cast<const uint8_t*>(fs.d_weak), S->h_weak.as<uint8_t>() + 4 * fs.off_tw,
                                   (int64_t)fs.C * 4};
                if (fs.dl > 0) tc[nt++] = CopyEnt{fs.d_strong, S->h_strong.as<uint8_t>() + fs.off_ts, (int64_t)fs.C * fs.dl};
                mt = std::max<int64_t>(mt, (int64_t)fs.C * 4);
                te[ntl++] = TableEnt{S->slots.as<unsigned long long>() + fs.off_ns, fs.d_weak, fs.ns - 1, fs.C};
            }
            RSH_BHIP(launch_copy_many(tc, nt, mt, st));
            RSH_BHIP(launch_table_clear(S->slots.as<unsigned long long>(), (uint64_t)tns, st));
            RSH_BHIP(launch_table_insert_many(te, ntl, (int32_t)maxC, st));
            CopyEnt* lc = S->h_ccopies.as<CopyEnt>() + NF;
            uint32_t nl = 0;
            int64_t mx = 0;
            for (FileScan& fs : files) {
                if (fs.done) continue;
                const int64_t nal = fs.be.na, nfl = std::min(fs.nf, nal);
                if (nfl > 0) lc[nl++] = CopyEnt{S->flags.as<uint8_t>() + fs.off_nf, S->h_fl.as<uint8_t>() + fs.off_nf, nfl};
                lc[nl++] = CopyEnt{S->src_weak.as<uint8_t>() + 4 * fs.off_na, S->h_aw.as<uint8_t>() + 4 * fs.off_na, nal * 4};
                if (fs.dl > 0)
                    lc[nl++] = CopyEnt{S->src_strong.as<uint8_t>() + fs.off_as, S->h_as.as<uint8_t>() + fs.off_as,
                                       nal * fs.dl};
                mx = std::max(mx, nal * 4);
            }
            RSH_BHIP(hipStreamWaitEvent(st, c->ev_spec, 0));
            RSH_BHIP(launch_copy_many(lc, nl, mx, st));
            RSH_BHIP(spin_sync(S, st));
            b.aligned.store(true);
            for (FileScan& fs : files) fs.be.head = false;
        }
        if (trace) {
            float kms = 0.f, wams = 0.f;
            if (S->ev_ch0 && S->ev_ch1) (void)hipEventElapsedTime(&kms, S->ev_ch0, S->ev_ch1);
            if (two_phase && S->ev_ch0 && S->ev_wa) (void)hipEventElapsedTime(&wams, S->ev_ch0, S->ev_wa);
            int64_t tsum = 0, esum = 0, dsum = 0, psum = 0, asum = 0, msum = 0;
            int32_t tmax = 0, emax = 0, fmax = 0;
            for (int32_t f = 0; f < NF; ++f) {
                tsum += co[f].tiles;
                msum += co[f].mapped;
                if (co[f].tiles > tmax) tmax = co[f].tiles, fmax = f;
                esum += co[f].events;
                dsum += co[f].digests;
                psum += co[f].md5c_valid;
                asum += co[f].aborted;
                emax = std::max<int32_t>(emax, (int32_t)co[f].events);
            }
            fprintf(stderr, "[rsh-batch] chain walks done at %.3f ms (walks %.3f ms, phase 0 %.3f ms; tiles %lld (%lld from the hit "
                    "map), max %d per file; events %lld, max %d; %lld windows digested, %lld files poisoned, %lld speculations "
                    "stopped at the prefix): %d of %d files left to the resolvers\n", ms_since(t0), kms, wams, (long long)tsum,
                    (long long)msum, tmax, (long long)esum, emax,
                    (long long)dsum, (long long)psum, (long long)asum, left, NF);
            const ChainOut& x = co[fmax];  // the walk with the most tiles: where its time went (10 ns ticks)
            for (int32_t f = 0; f < NF; ++f)  // the walks that left their files to the resolvers: where and why
                if (co[f].status != CHAIN_DONE)
                    fprintf(stderr, "[rsh-batch]   file %d: left at s %lld (why %d, events %lld, tiles %d, poisoned %d, searched to "
                            "%lld, phase 1 %d, walk %.1f us)\n", f, (long long)co[f].s, co[f].why, (long long)co[f].events,
                            co[f].tiles, co[f].md5c_valid, (long long)co[f].clear_to, co[f].spec_full, co[f].t_total / 100.0);
            fprintf(stderr, "[rsh-batch]   file %d: walk %.1f us = tiles %.1f (table checks %.1f; %d of %d tiles from the hit map,"
                    " the first at tile %d) + events %.1f (buckets %.1f; %d digests: %.1f) + key set %.1f + steps (1)/(1') %.1f +"
                    " event drains %.1f + other\n", fmax, x.t_total / 100.0,
                    x.t_tiles / 100.0, x.t_check / 100.0, x.mapped, x.tiles, x.first_mapped, x.t_event / 100.0,
                    x.t_evb / 100.0, x.digests, x.t_digest / 100.0, x.t_kset / 100.0, x.t_chain / 100.0, x.t_drain / 100.0);
            if (S->chain_help.p && two_phase) {  // the map's helpers (device state of the last phase-0 launch)
                std::vector<ChainHelp> hh((size_t)NF);
                if (hipMemcpy(hh.data(), S->chain_help.p, (size_t)NF * sizeof(ChainHelp), hipMemcpyDeviceToHost) == hipSuccess) {
                    int64_t segs = 0, joins = 0, files_helped = 0;
                    for (const ChainHelp& q : hh) {
                        segs += q.mapped;
                        joins += q.joins;
                        files_helped += q.joins > 0;
                    }
                    const ChainHelp& q = hh[(size_t)fmax];
                    fprintf(stderr, "[rsh-batch]   hit map: %lld segments mapped over %lld files (%lld key sets built); file %d: %d "
                            "segments (%d whole), %d key sets (%.1f us each), claims %d of %d, first whole segment %.1f us after "
                            "the walk's start\n", (long long)segs, (long long)files_helped, (long long)joins, fmax, q.mapped,
                            q.whole, q.joins, q.joins ? q.t_kset / 100.0 / q.joins : 0.0, q.claim, q.nseg,
                            q.t_first == INT64_MAX ? -1.0 : (q.t_first - q.t_start) / 100.0);
                }
            }
        }
    }
    if (tentative) {
        for (int32_t f = 0; f < NF; ++f) {
            FileScan& fs = files[(size_t)f];
            const int64_t a = lead_at[(size_t)f], nl = lead_at[(size_t)f + 1] - a;
            int64_t lead = 0;
            while (lead < nl && lead_w[a + lead] == fs.table.weak[lead]) ++lead;
            fs.wait_spec = nl > 0 && lead == nl && (nl >= kLeadWindows || nl == fs.nf);
            nwait += fs.wait_spec;
        }
        if (nwait > 0) {
            spec_rc = launch_spec();
            if (spec_rc != RSH_OK) return spec_rc;
            spec_launched = true;
        } else {  // no file qualifies: stop it (every group polls its file's word); the deferred launch stays
            RSH_BHIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(S->file_abort), gen, (size_t)NF, st));
            RSH_BHIP(hipStreamWaitEvent(st, S->ev_scopy, 0));
            gen = c->next_gen();
            k1_launched = false;
        }
        if (trace) fprintf(stderr, "[rsh-batch] lead check: %d of %d files wait for the speculation\n", nwait, NF);
    }
    if (early_spec && !wait_spec) {
        spec_rc = launch_spec();  // the tail (flags, downloads) behind the K1 already running
        if (spec_rc != RSH_OK) return spec_rc;
        spec_launched = true;
    }
    if (wait_spec) {
        spec_rc = launch_spec();
        if (spec_rc != RSH_OK) return spec_rc;
        spec_launched = true;
        RSH_BHIP(hipEventSynchronize(c->ev_spec));
        if (trace) fprintf(stderr, "[rsh-batch] speculation landed at %.3f ms\n", ms_since(t0));
        b.landed.store(true);
        b.aligned.store(true);
        for (FileScan& fs : files) fs.be.head = false;
    }

    RoundCtl ctl;
    ctl.launch_spec = launch_spec;
    ctl.spec_launched = &spec_launched;
    ctl.spec_rc = &spec_rc;
    ctl.defer_rounds = defer_rounds;
    ctl.k1_launched = k1_launched;
    ctl.gen = gen;
    ctl.trace = trace;
    ctl.t0 = t0;
    int rounds = 0;
    const hipError_t err = run_resolvers(c, S, bp, files, st, ctl, &rounds);
    const double rounds_end_ms = ms_since(t0);
    const double resolve_ms = ms_since(t0) - setup_ms;
    if (trace) {
        HostTimes tt;
        for (const HostTimes& x : b.times) {
            tt.bucket_ms += x.bucket_ms;
            tt.sort_ms += x.sort_ms;
            tt.dkeys_ms += x.dkeys_ms;
            tt.md5_ms += x.md5_ms;
        }
        fprintf(stderr, "[rsh-batch] host totals (cumulative per thread): bucket %.3f sort %.3f dkeys %.3f md5 %.3f ms\n",
                tt.bucket_ms, tt.sort_ms, tt.dkeys_ms, tt.md5_ms);
    }
    if (trace)
        fprintf(stderr, "[rsh-batch] %d files: enqueued %.3f, tables+hashes ready %.3f, rounds done %.3f, joined %.3f ms\n",
                NF, enq_ms, setup_ms, rounds_end_ms, ms_since(t0));

    if (spec_launched) {
        // every resolver finished before the speculation's K1 did: stop it.  (Once its flags have landed the
        // K1 is done; the sums' download may still run on the aux stream, which the next call's work on that
        // stream follows anyway.)
        if (!b.landed.load() && hipEventQuery(c->ev_flags) == hipSuccess) b.landed.store(true);
        if (!b.landed.load()) {
            // the batched K1's groups poll their own file's word (K1Group::abort), not the launch's: stop
            // every file not cancelled yet (those resolved in the last round included)
            for (int32_t f = 0; f < NF; ++f) {
                FileScan& fs = files[(size_t)f];
                if (fs.cancelled) continue;
                fs.cancelled = true;
                RSH_BHIP(hipStreamWriteValue32(st, S->file_abort + f, (uint32_t)gen, 0));
            }
            if (trace) fprintf(stderr, "[rsh-batch] scan done before the speculation landed: stopped\n");
            RSH_BHIP(hipStreamWriteValue32(st, c->abort_word, (uint32_t)gen, 0));
            RSH_BHIP(hipStreamWaitEvent(st, c->ev_spec, 0));
        }
    }
    if (spec_rc != RSH_OK) return spec_rc;
    if (err != hipSuccess) return RSH_E_DEVICE;

    // the events to the callers' buffers: on several threads when there are many (config 4's 50%-modified form
    // returns ~1650 events per file, 6.7 MB for 128 files)
    std::vector<int32_t> copy_files;
    int64_t copy_bytes = 0;
    for (int32_t f = 0; f < NF; ++f) {
        FileScan& fs = files[(size_t)f];
        rsh_scan_job& j = jobs[fs.job];
        j.literal = fs.res.literal;
        j.matched = fs.res.matched;
        j.n_ev = fs.dev_ev ? fs.dev_n : (int64_t)fs.res.ev.size();
        if (j.n_ev > j.ev_cap || (!j.ev && j.n_ev > 0)) {
            j.status = RSH_E_NOSPACE;
        } else {
            if (j.n_ev > 0) {
                copy_files.push_back(f);
                copy_bytes += j.n_ev * (int64_t)sizeof(rsh_event);
            }
            j.status = RSH_OK;
        }
    }
    auto copy_range = [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            FileScan& fs = files[(size_t)copy_files[i]];
            rsh_scan_job& j = jobs[fs.job];
            memcpy(j.ev, fs.dev_ev ? fs.dev_ev : fs.res.ev.data(), (size_t)j.n_ev * sizeof(rsh_event));
        }
    };
    const int nct = copy_bytes > (1 << 20) ? std::min<int>(8, std::max(1, call_cores())) : 1;
    if (nct > 1 && copy_files.size() > 1) {  // on the context's persistent pool (HostPool, batch.h)
        const size_t per = (copy_files.size() + (size_t)nct - 1) / (size_t)nct;
        const int parts = (int)((copy_files.size() + per - 1) / per);
        S->pool.ensure(parts - 1);
        const std::function<void(int)> part = [&](int k) {
            copy_range((size_t)k * per, std::min(copy_files.size(), (size_t)(k + 1) * per));
        };
        S->pool.run(parts, part);
    } else {
        copy_range(0, copy_files.size());
    }
    for (FileScan& fs : files) {
        if (agg) {
            const rsh_scan_stats& s = fs.res.stats;
            agg->chain_matches += s.chain_matches;
            agg->events += s.events;
            agg->host_md5_windows += s.host_md5_windows;
            agg->flushes += s.flushes;
            agg->table_ms += s.table_ms + fs.table.sort_ms;
            int64_t spec_bytes = (spec_launched && b.landed.load() && !fs.cancelled) ? fs.n : 0;
            if (spec_bytes > 0 && fs.be.na < fs.na)  // a two-phase file that stopped in its prefix: the prefix K1,
                spec_bytes = std::min<int64_t>(fs.n, fs.be.na * fs.B) + (skip_rest ? 0 : fs.lane_b_bytes);  // + phase 1's lane chunks
            agg->device_bytes += fs.be.bytes_read + spec_bytes;
            agg->phase_matches += s.phase_matches;
        }
    }
    if (agg) {
        agg->probe_launches += rounds;  // one batched launch set per round
        agg->device_ms += setup_ms;
        agg->resolver_ms += resolve_ms;
        agg->speculation_aborted = spec_launched ? (b.landed.load() ? 0 : 1) : 2;
    }
    return RSH_OK;
}

}  // namespace
}  // namespace batch
}  // namespace rsh

using namespace rsh;

namespace rsh {
using namespace batch;

// rsh_ctx_create (scan.cpp ctx_warm): the batched scan's and the batched Generator's state pre-sized for a segment of
// `nfiles` files of n bytes at block length B, digest length dl -- the sizes scan_batch and block_sums_batch_claimed
// grow them to for that segment (the same formulas, mirrored here) -- so that a context's first segment scan
// allocates nothing (~11 ms of pinned allocations on config 4's first call).  Option batch_warm
// sets nfiles (0: none); the shape is config 4's (128 MiB files, B 8192, dl 4): ~50 MiB pinned, ~0.25 GiB of HBM.
hipError_t batch_warm(rsh_ctx* c, int32_t nfiles, int64_t n, int64_t B, int32_t dl) {
    if (nfiles <= 0) return hipSuccess;
    BatchState* S = state_of(c);
    if (!S) return hipErrorOutOfMemory;
    const int64_t NF = std::min<int64_t>(nfiles, kMaxLive);
    const int64_t C = (n + B - 1) / B, na = C, nf = C, ns = pow2_at_least(2 * (uint64_t)C + 2);
    const int64_t tw = NF * C, ts = NF * C * dl, tna = NF * na, tas = NF * na * dl, tnf = NF * nf, tns = NF * ns,
                  thit = NF * pad16(16 + B), tw0 = NF * pad16(std::min<int64_t>(B, n));
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t x) {
        if (e == hipSuccess) e = x;
    };
    // scan_batch: the per-file tables, sums and descriptors
    ok(S->h_weak.ensure((size_t)tw * 4 + 4));
    ok(S->h_strong.ensure((size_t)ts + 1));
    ok(S->slots.ensure((size_t)tns * 8));
    ok(S->src_weak.ensure((size_t)tna * 4));
    ok(S->src_strong.ensure((size_t)tas + 1));
    ok(S->flags.ensure((size_t)tnf + 1));
    ok(S->haw.ensure((size_t)tna * 4));
    ok(S->h_aw.ensure((size_t)tna * 4));
    ok(S->h_as.ensure((size_t)tas + 1));
    ok(S->h_fl.ensure((size_t)tnf + 1));
    ok(S->h_files.ensure((size_t)NF * sizeof(ScanFile)));
    ok(S->h_hit.ensure((size_t)thit));
    ok(S->h_win0.ensure((size_t)tw0));
    ok(S->first.ensure((size_t)NF * sizeof(ProbeOut)));
    ok(S->h_first.ensure((size_t)NF * sizeof(ProbeOut)));
    ok(S->bucket.ensure((size_t)NF * HIT_BUCKET_INTS * 4));
    ok(S->h_bucket.ensure((size_t)NF * HIT_BUCKET_INTS * 4));
    ok(S->h_copies.ensure((size_t)2 * NF * sizeof(CopyEnt)));
    ok(S->h_ccopies.ensure((size_t)NF * sizeof(CopyEnt) + (size_t)3 * NF * sizeof(CopyEnt)));
    ok(S->h_tabents.ensure((size_t)NF * sizeof(TableEnt)));
    ok(S->h_flagents.ensure((size_t)NF * sizeof(FlagEnt)));
    ok(S->h_flagents_a.ensure((size_t)NF * sizeof(FlagEnt)));
    ok(S->ensure_file_abort(NF));
    const int64_t nlead_all = NF * std::min<int64_t>(kLeadWindows, nf);
    ok(S->h_lead.ensure((((size_t)(nlead_all + 1) * 4 + 63) & ~(size_t)63) + (size_t)(nlead_all + 1) * sizeof(GatherEnt)));
    // the K1 descriptors of both phases (planned from the shapes alone: the data pointers only set the alignment)
    std::vector<K1File> kf((size_t)NF), ka((size_t)NF), kb((size_t)NF);
    const int64_t P = 16 * std::max<int64_t>(1, kWaveSlots / NF), na_a = std::min(na, P);
    const uint8_t* const al = reinterpret_cast<const uint8_t*>(uintptr_t{4096});  // 128-B aligned stand-in
    for (int64_t f = 0; f < NF; ++f) {
        kf[(size_t)f] = K1File{al, n, (uint32_t)B, (uint32_t)dl, (uint32_t)na, nullptr, nullptr};
        ka[(size_t)f] = K1File{al, std::min<int64_t>(n, na_a * B), (uint32_t)B, (uint32_t)dl, (uint32_t)na_a, nullptr, nullptr};
        kb[(size_t)f] = K1File{al, n - na_a * B, (uint32_t)B, (uint32_t)dl, (uint32_t)(na - na_a), nullptr, nullptr};
    }
    std::vector<K1Plan> plans, pa, pb;
    std::vector<K1Lane> lanes, la, lb;
    int al0 = 16, al1 = 16, al2 = 16;
    bool p0 = tail_gather_on(), p1 = tail_gather_on(), p2 = tail_gather_on();
    const uint32_t ng = plan_block_sums_files(kf.data(), (int32_t)NF, &plans, &lanes, &al0, &p0);
    const uint32_t nga = plan_block_sums_files(ka.data(), (int32_t)NF, &pa, &la, &al1, &p1);
    const uint32_t ngb = na > na_a ? plan_block_sums_files(kb.data(), (int32_t)NF, &pb, &lb, &al2, &p2) : 0;
    ok(S->k1_groups.ensure(((size_t)std::max(ng, nga + ngb) + 1) * sizeof(K1Group)));
    ok(S->k1_plans.ensure((std::max(plans.size(), pa.size() + pb.size()) + 1) * sizeof(K1Plan)));
    ok(S->k1_lanes.ensure((std::max(lanes.size(), la.size() + lb.size()) + 1) * sizeof(K1Lane)));
    ok(S->h_sgroups.ensure((std::max(plans.size(), pa.size() + pb.size()) + 1) * sizeof(K1Plan)));
    ok(S->h_slanes.ensure((std::max(lanes.size(), la.size() + lb.size()) + 1) * sizeof(K1Lane)));
    // the chain walks: chunk indexes, descriptors, events, the phase-0 hit map
    const int64_t kChainEvents = std::clamp<int64_t>(kChainEventBytes / (NF * (int64_t)sizeof(rsh_event)), 256, kChainEventsMax);
    ok(S->kslots.ensure(kslots_bytes(tns, tw)));
    ok(S->h_kents.ensure((size_t)NF * sizeof(ChunkIndexEnt)));
    ok(S->h_chain.ensure((size_t)NF * sizeof(ChainFile)));
    ok(S->h_chain_out.ensure((size_t)NF * sizeof(ChainOut)));
    ok(S->h_chain_ev.ensure((size_t)(NF * kChainEvents) * sizeof(rsh_event)));
    const bool wide = B >= 512 && B % 32 == 0 && CHAIN_TILE / B + 2 <= CHAIN_SEGS;
    const int64_t words = wide && na > na_a ? NF * ((std::min<int64_t>(na_a * B, n - B + 1) + 31) / 32) : 0;
    if (words > 0 && words * 8 <= opt(OPT_CHAIN_MAP_BYTES) && (size_t)words * 8 > S->chain_map.cap) {
        ok(S->chain_map.ensure((size_t)words * 8));
        if (e == hipSuccess) ok(hipMemset(S->chain_map.p, 0, S->chain_map.cap));  // no stale generation
    }
    ok(S->chain_help.ensure((size_t)NF * sizeof(ChainHelp)));
    ok(S->h_chain_help.ensure((size_t)NF * sizeof(ChainHelp)));
    ok(S->h_early.ensure(4096));
    S->pool.ensure(7);  // the events' copy threads (scan_batch: up to 8 parts, the caller takes one)
    // the resolver rounds' staging (serve_round), at PinnedBuf's least size: ~40 us per pinned allocation
    for (PinnedBuf* pb : {&S->h_fjobs, &S->h_fout, &S->h_rcp, &S->h_req, &S->h_gw, &S->h_gb, &S->h_ow, &S->h_ob, &S->h_win,
                          &S->h_dkeys})
        ok(pb->ensure(64 << 10));
    // ... and a stale digest's batched flush chain at its largest (4096 intervals: its gathers, intervals, tiles and
    // segments; a staging buffer that grows frees the old one first, ~0.3 ms on the first call)
    for (PinnedBuf* pb : {&S->h_fgw, &S->h_iv, &S->h_tiles, &S->h_segs, &S->h_ptiles}) ok(pb->ensure(512 << 10));
    for (DevBuf* db : {&S->fc_dev, &S->partials, &S->dslots, &S->d_probe}) ok(db->ensure(64 << 10));
    for (hipEvent_t* ev : {&S->ev_fk, &S->ev_fa, &S->ev_scopy, &S->ev_sync, &S->ev_gcopy})
        if (!*ev) ok(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    if (!S->ev_wa) ok(hipEventCreate(&S->ev_wa));
    // block_sums_batch_claimed: the Generator's descriptors
    ok(S->g_groups.ensure(((size_t)ng + 1) * sizeof(K1Group)));
    ok(S->g_plans.ensure((plans.size() + 1) * sizeof(K1Plan)));
    ok(S->g_lanes.ensure((lanes.size() + 1) * sizeof(K1Lane)));
    ok(S->h_ggroups.ensure((plans.size() + 1) * sizeof(K1Plan)));
    ok(S->h_glanes.ensure((lanes.size() + 1) * sizeof(K1Lane)));
    return e;
}

// rsh_block_sums_batch_device with the context already claimed by the caller (segment.cpp builds the host forms
// on it).
int block_sums_batch_claimed(rsh_ctx* ctx, const rsh_block_job* jobs, int32_t njobs, const uint8_t seed[4]) {
    if (!ctx || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    std::vector<K1File> files;
    for (int32_t i = 0; i < njobs; ++i) {
        const rsh_block_job& j = jobs[i];
        const int rc = check_generator_header(j.n, &j.h);
        if (rc != RSH_OK) return rc;
        if (j.h.chunk_count == 0) continue;
        if (!j.d_data || !j.d_weak || (!j.d_strong && j.h.digest_length > 0)) return RSH_E_INVAL;
        files.push_back(K1File{static_cast<const uint8_t*>(j.d_data), j.n, (uint32_t)j.h.block_length,
                               (uint32_t)j.h.digest_length, (uint32_t)j.h.chunk_count, static_cast<int32_t*>(j.d_weak),
                               static_cast<uint8_t*>(j.d_strong)});
    }
    if (files.empty()) return RSH_OK;
    BatchState* S = state_of(ctx);
    if (!S) return RSH_E_NOMEM;
    RSH_BHIP(hipSetDevice(ctx->device));
    std::vector<K1Plan> plans;
    std::vector<K1Lane> lanes;
    int lane_align = 16;
    bool partial = tail_gather_on();
    const uint32_t ngroups =
        plan_block_sums_files(files.data(), (int32_t)files.size(), &plans, &lanes, &lane_align, &partial);
    RSH_BHIP(S->g_groups.ensure(((size_t)ngroups + 1) * sizeof(K1Group)));
    RSH_BHIP(S->g_plans.ensure((plans.size() + 1) * sizeof(K1Plan)));
    RSH_BHIP(S->g_lanes.ensure((lanes.size() + 1) * sizeof(K1Lane)));
    if (!S->ev_gcopy) RSH_BHIP(hipEventCreateWithFlags(&S->ev_gcopy, hipEventDisableTiming));
    if (S->gcopy_pending) RSH_BHIP(hipEventSynchronize(S->ev_gcopy));  // the previous call's upload is done
    S->gcopy_pending = false;
    RSH_BHIP(S->h_ggroups.ensure((plans.size() + 1) * sizeof(K1Plan)));
    RSH_BHIP(S->h_glanes.ensure((lanes.size() + 1) * sizeof(K1Lane)));
    if (!plans.empty()) {
        memcpy(S->h_ggroups.p, plans.data(), plans.size() * sizeof(K1Plan));
        RSH_BHIP(hipMemcpyAsync(S->g_plans.p, S->h_ggroups.p, plans.size() * sizeof(K1Plan), hipMemcpyHostToDevice,
                                ctx->stream));
    }
    if (!lanes.empty()) {
        memcpy(S->h_glanes.p, lanes.data(), lanes.size() * sizeof(K1Lane));
        RSH_BHIP(hipMemcpyAsync(S->g_lanes.p, S->h_glanes.p, lanes.size() * sizeof(K1Lane), hipMemcpyHostToDevice,
                                ctx->stream));
    }
    RSH_BHIP(hipEventRecord(S->ev_gcopy, ctx->stream));
    S->gcopy_pending = true;
    RSH_BHIP(launch_expand_groups(S->g_plans.as<K1Plan>(), (uint32_t)plans.size(), ngroups, S->g_groups.as<K1Group>(),
                                  ctx->stream));
    RSH_BHIP(launch_block_sums_batch(S->g_groups.as<K1Group>(), ngroups, S->g_lanes.as<K1Lane>(),
                                     (uint32_t)lanes.size(), lane_align, seed_word(seed), ctx->stream, nullptr, 0,
                                     partial));
    return RSH_OK;
}

// rsh_match_scan_batch_device with the context already claimed by the caller.
int match_scan_batch_claimed(rsh_ctx* ctx, rsh_scan_job* jobs, int32_t njobs, const uint8_t seed[4],
                             rsh_scan_stats* stats) {
    if (!ctx || !seed || njobs < 0 || (njobs > 0 && !jobs)) return RSH_E_INVAL;
    if (stats) *stats = rsh_scan_stats{};
    std::vector<int32_t> scan;
    for (int32_t i = 0; i < njobs; ++i) {
        rsh_scan_job& j = jobs[i];
        j.n_ev = j.literal = j.matched = 0;
        j.status = RSH_OK;
        if (j.n < 0) {
            j.status = RSH_E_INVAL;
            continue;
        }
        const int v = rsh_header_validate(&j.h);
        if (v != RSH_OK) {
            j.status = v;
            continue;
        }
        if (j.h.block_length == 0 || j.n == 0) {  // new file (skipMatchSendData) or empty source
            ResolveResult r;
            if (j.h.block_length == 0) skip_events(j.n, &r);
            j.literal = r.literal;
            j.n_ev = (int64_t)r.ev.size();
            if (j.n_ev > j.ev_cap || (!j.ev && j.n_ev > 0)) j.status = RSH_E_NOSPACE;
            else if (j.n_ev > 0) memcpy(j.ev, r.ev.data(), r.ev.size() * sizeof(rsh_event));
            continue;
        }
        if (!j.d_src || (j.h.chunk_count > 0 && (!j.d_weak || (!j.d_strong && j.h.digest_length > 0)))) {
            j.status = RSH_E_INVAL;
            continue;
        }
        if ((j.n + j.h.block_length - 1) / j.h.block_length > 2147483647LL) {
            j.status = RSH_E_OVERFLOW;
            continue;
        }
        scan.push_back(i);
    }
    if (!scan.empty()) {
        // a failing call leaves no file it did not finish at RSH_OK: that file and every later one carry its code
        // (a caller that trusts per-file statuses must never read zeros as results)
        auto fail_from = [&](size_t k, int rc) {
            for (size_t q = k; q < scan.size(); ++q) jobs[scan[q]].status = rc;
            return rc;
        };
        if (hipSetDevice(ctx->device) != hipSuccess) return fail_from(0, RSH_E_DEVICE);
        for (size_t k = 0; k < scan.size(); k += kMaxLive) {
            const std::vector<int32_t> part(scan.begin() + (ptrdiff_t)k,
                                            scan.begin() + (ptrdiff_t)std::min(scan.size(), k + kMaxLive));
            const int rc = scan_batch(ctx, jobs, part, seed, stats);
            if (rc != RSH_OK) return fail_from(k, rc);
        }
    }
    for (int32_t i = 0; i < njobs; ++i)
        if (jobs[i].status != RSH_OK) return jobs[i].status;
    return RSH_OK;
}

}  // namespace rsh

extern "C" {

int rsh_block_sums_batch_device(rsh_ctx* ctx, const rsh_block_job* jobs, int32_t njobs, const uint8_t seed[4]) {
    if (!ctx) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    return rsh::block_sums_batch_claimed(ctx, jobs, njobs, seed);
}

int rsh_match_scan_batch_device(rsh_ctx* ctx, rsh_scan_job* jobs, int32_t njobs, const uint8_t seed[4],
                                rsh_scan_stats* stats) {
    if (!ctx) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    return rsh::match_scan_batch_claimed(ctx, jobs, njobs, seed, stats);
}

}  // extern "C"
