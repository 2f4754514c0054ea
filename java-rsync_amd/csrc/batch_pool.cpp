// batch_pool.cpp -- the batched scan's resolver pool: the resolvers left after the chain walks run as fibers on a
// few worker threads (one per host core of the call, at most kMaxWorkers), their device questions become requests
// (BatchBackend, Req), and the calling thread serves them one round at a time -- one launch per kind and one stream
// synchronisation per round for the whole segment (serve_round).  The scheduler's invariants are at the top of
// batch.h.  Sender.java:1235-1327 per file (resolver.cpp), Sender.sendFiles :1098-1148 for the segment.
#include "batch.h"

namespace rsh {

// The cores this process may use: its affinity mask, capped by a cgroup CPU quota (cgroup v2 cpu.max,
// "quota period"; containers often see every CPU of the machine in the mask but get a few cores' worth of
// time).  More spinning workers than that get throttled by the scheduler for whole periods.
int host_cores() {
    if (const int64_t o = opt(OPT_HOST_CORES); o > 0) return (int)o;  // explicit override (options.h)
    static const int v = [] {
        int n = 8;
        cpu_set_t cpus;
        if (sched_getaffinity(0, sizeof(cpus), &cpus) == 0) n = CPU_COUNT(&cpus);
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            long long period = 0;
            if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
                const long long quota = atoll(q);
                if (quota > 0) n = std::min<int>(n, (int)std::max<long long>(1, quota / period));
            }
            fclose(f);
        }
        return n;
    }();
    return v;
}

namespace batch {

// A resolver fiber: head mode until the batched speculation lands, then resume with it (resolve_run is
// resumable); returning switches to uc_link (its worker).
void fiber_main(uint32_t hi, uint32_t lo) {
    FileScan& fs = *reinterpret_cast<FileScan*>(((uintptr_t)hi << 32) | lo);
    BatchBackend& be = fs.be;
    Batch& b = *be.b;
    // small tables are sorted up front, here on the worker threads (in parallel across files): a segment's
    // resolvers would otherwise spend their first rounds in linear bucket scans before the lazy sort
    if (fs.C <= kEagerSortChunks) fs.table.build();
    if (fs.wait_spec) {  // a run of aligned matches from the start: nothing to do until the speculation lands
        fs.req = Req{};
        fs.req.kind = Req::WAIT;
        b.post(fs);
        be.head = false;
    }
    while (!resolve_run(fs.n, fs.table, be, &fs.rs, &fs.res,
                        [&] { return be.head && b.landed.load(std::memory_order_acquire); }))
        be.head = false;
    fs.done = true;
}

void BatchBackend::weak_many(const int64_t* pos, int64_t count, int32_t* out) {
    if (count <= 0) return;
    if (count == 1 && pos[0] == t_pos) {  // came back with (or derived from) a probe result
        out[0] = t_val;
        return;
    }
    bytes_read += count * B;
    FileScan& fs = scan_of(b, f);
    fs.req = Req{};
    fs.req.kind = Req::WEAK;
    fs.req.pos = pos;
    fs.req.count = count;
    fs.req.out_w = out;
    b->post(fs);
}

void BatchBackend::bytes_many(const int64_t* pos, int64_t count, uint8_t* out) {
    if (count <= 0) return;
    bytes_read += count;
    FileScan& fs = scan_of(b, f);
    fs.req = Req{};
    fs.req.kind = Req::BYTES;
    fs.req.pos = pos;
    fs.req.count = count;
    fs.req.out_b = out;
    b->post(fs);
}

void BatchBackend::flush_gather(const int64_t* tpos, int64_t nt, int32_t* tv, const int64_t* bpos, int64_t nb,
                                uint8_t* bv) {
    if (nt <= 0 || nb <= 0) {
        ScanBackend::flush_gather(tpos, nt, tv, bpos, nb, bv);
        return;
    }
    bytes_read += nt * B + nb;
    FileScan& fs = scan_of(b, f);
    fs.req = Req{};
    fs.req.kind = Req::FLUSH;
    fs.req.pos = tpos;
    fs.req.count = nt;
    fs.req.out_w = tv;
    fs.req.pos2 = bpos;
    fs.req.count2 = nb;
    fs.req.out_b2 = bv;
    b->post(fs);
}

// bytes copied per window request (A/B option batch_readahead; never less than the window).  Off by
// default: on config 4 it cut the rounds from 23 to 18, but the head-mode rounds it removed were cheap
// window copies and the probes left in their place wait behind the speculation K1
int64_t readahead_bytes() { return std::max<int64_t>(0, opt(OPT_BATCH_READAHEAD)); }

void BatchBackend::md5_at(int64_t p, uint8_t out[16]) {
    const int64_t w = std::min<int64_t>(B, n - p);
    const uint8_t* src = nullptr;
    if (p == 0 && win0) src = win0;                 // copied to the host before the first round
    else {
        for (int k = 0; k < HIT_WINDOWS; ++k)
            if (p == win_pos[k]) src = hit + 16 + (int64_t)k * B;  // came back with the probe result
    }
    if (!src && pf_pos >= 0 && p >= pf_pos && p + w <= pf_pos + (int64_t)pf.size()) src = pf.data() + (p - pf_pos);
    if (!src) {
        FileScan& fs = scan_of(b, f);
        const int64_t ext = std::min<int64_t>(std::max<int64_t>(w, readahead_bytes()), n - p);
        fs.req = Req{};
        fs.req.kind = Req::WIN;
        fs.req.p = p;
        fs.req.w = ext;
        bytes_read += ext;
        b->post(fs);
        src = fs.req.win;
        if (ext > w) {  // keep the read-ahead (the round's window buffer is reused by the next round)
            pf.assign(src, src + ext);
            pf_pos = p;
            src = pf.data();
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    HostMd5 h;  // one serial chain per window: on this file's host thread, beside the other files' work
    h.update(src, (size_t)w);
    h.update(seed, 4);
    h.final(out);
    host_times().md5_ms += ms_since(t0);
}

int64_t BatchBackend::first_hit(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys) {
    ProbeInterval one;
    if (count == 1) {  // answered by the previous probe's hit list, or cut to its unprobed part
        int64_t p = -1, a2 = iv[0].a;
        int32_t T = 0;
        if (cache.lookup(iv[0], keys, &p, &T, &a2)) {
            if (p >= 0) {
                t_pos = p;
                t_val = T;
            }
            return p;
        }
        one = iv[0];
        one.a = a2;
        iv = &one;
    }
    bytes_read += probe_bytes(iv, count, B);
    FileScan& fs = scan_of(b, f);
    fs.req = Req{};
    fs.req.kind = Req::PROBE;
    fs.req.iv = iv;
    fs.req.niv = count;
    fs.req.keys = keys;
    fs.req.head = head;
    b->post(fs);
    return probe_answer(iv, count, keys);
}

// the answer of a PROBE / FCHAIN round: the hit cache, the windows and buckets that came with it
int64_t BatchBackend::probe_answer(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys) {
    FileScan& fs = scan_of(b, f);
    const int64_t p = fs.req.result;
    if (count == 1 && fs.req.out) cache.fill(iv[0], keys, *fs.req.out, n - B);
    else if (fs.req.out) cache.fill_batch(iv, count, keys, *fs.req.out, n - B);
    else cache.valid = false;
    if (p < 0) return -1;
    window_slots(*fs.req.out, 1, win_pos);
    t_pos = p;
    t_val = *reinterpret_cast<const int32_t*>(hit);
    prime_from_probe(*table, *fs.req.out, bucket);
    return p;
}

int64_t BatchBackend::flush_probe(const ProbeInterval* pre, int64_t npre, const FlushChain& q,
                                  std::vector<FlushStep>* steps, std::vector<ProbeInterval>* ivs,
                                  const std::vector<int32_t>* keys) {
    flush_intervals(q, steps, ivs);
    if (ivs->empty()) return ScanBackend::flush_probe(pre, npre, q, steps, ivs, keys);  // (no interval opens)
    std::vector<int64_t> tpos, bpos;
    flush_positions(q, &tpos, &bpos);
    std::vector<ProbeInterval> all(pre, pre + npre);
    all.insert(all.end(), ivs->begin(), ivs->end());
    std::vector<uint32_t> out((size_t)(2 * q.K));
    bytes_read += probe_bytes(all.data(), (int64_t)all.size(), B) + (int64_t)tpos.size() * B + (int64_t)bpos.size();
    FileScan& fs = scan_of(b, f);
    fs.req = Req{};
    fs.req.kind = Req::FCHAIN;
    fs.req.pos = tpos.data();
    fs.req.count = (int64_t)tpos.size();
    fs.req.pos2 = bpos.data();
    fs.req.count2 = (int64_t)bpos.size();
    fs.req.iv = all.data();
    fs.req.niv = (int64_t)all.size();
    fs.req.keys = keys;
    fs.req.head = head;
    fs.req.fchain = q;
    fs.req.npre = npre;
    fs.req.chain_out = out.data();
    b->post(fs);
    for (size_t i = 0; i < steps->size(); ++i) {
        (*steps)[i].elo = out[2 * i];
        (*steps)[i].ehi = out[2 * i + 1];
        if (i < ivs->size()) {
            (*ivs)[i].e_lo = all[(size_t)npre + i].e_lo = out[2 * i];
            (*ivs)[i].e_hi = all[(size_t)npre + i].e_hi = out[2 * i + 1];
        }
    }
    return probe_answer(all.data(), (int64_t)all.size(), keys);
}

// One round: answer every pending request of the batch.  Returns a HIP error (then every request is
// answered with "nothing": the resolvers run to completion on garbage and the batch reports the error).
// Wait for an event by polling it: the resolver rounds sit on this latency path, and a blocking wait can sleep past
// the completion (the runtime's yield) -- each round's hand-off back to the host is ~10-50 us of the step otherwise.
hipError_t spin_event(hipEvent_t ev) {
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        _mm_pause();
    }
}
// ... and for everything enqueued on st so far
hipError_t spin_sync(BatchState* S, hipStream_t st) {
    if (!S->ev_sync) {
        const hipError_t e = hipEventCreateWithFlags(&S->ev_sync, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    const hipError_t e = hipEventRecord(S->ev_sync, st);
    return e != hipSuccess ? e : spin_event(S->ev_sync);
}

hipError_t serve_round(rsh_ctx* c, BatchState* S, std::vector<FileScan>& files, const std::vector<int32_t>& pend,
                       hipStream_t st) {
    std::vector<GatherEnt> gw, gb;
    std::vector<CopyEnt> copies;
    std::vector<ProbeIv> ivs;
    std::vector<ProbeTile> tiles;
    std::vector<ProbeSeg> segs;
    std::vector<PartialTile> ptiles;
    std::vector<int32_t> preq;
    std::vector<int64_t> gw_at(files.size(), -1), gb_at(files.size(), -1), win_at(files.size(), -1);
    int64_t win_bytes = 0, max_win = 0;
    int32_t max_C = 0;
    std::vector<uint64_t> dkeys;  // host-built probe hashes of stale-digest key sets
    struct DkeyTab {
        int32_t f;
        int64_t off;
        uint32_t mask;
    };
    std::vector<DkeyTab> dtabs;

    ScanFile* F = S->h_files.as<ScanFile>();
    // FCHAIN: the chains' gathers (into device memory) and the place of each chain's outputs in h_fout
    std::vector<GatherEnt> fw, fb;
    std::vector<int64_t> fw_at(files.size(), -1), fb_at(files.size(), -1), fo_at(files.size(), -1);
    int64_t nfout = 0;
    // a PROBE (or FCHAIN) request's intervals, tiles and key set into this round's launch
    auto plan_probe = [&](int32_t f) {
        FileScan& fs = files[(size_t)f];
        Req& r = fs.req;
        BatchBackend& be = fs.be;
        F[f].aligned_weak = r.head ? S->haw.as<int32_t>() + fs.off_na : S->src_weak.as<int32_t>() + fs.off_na;
        F[f].slots = S->slots.as<unsigned long long>() + fs.off_ns;
        F[f].mask = fs.ns - 1;
        F[f].nsmall = 0;
        if (r.keys && !r.keys->empty() && r.keys->size() <= (size_t)PROBE_SMALL_KEYS) {  // compared in registers
            F[f].nsmall = (int32_t)r.keys->size();
            for (size_t j = 0; j < r.keys->size(); ++j) F[f].small[j] = (uint32_t)(*r.keys)[j];
        } else if (r.keys) {  // stale digest: only its chunks' keys (a handful), hashed here
            const uint32_t nsl = pow2_at_least(2 * r.keys->size() + 2);
            const int64_t off = (int64_t)dkeys.size();
            dkeys.resize(dkeys.size() + nsl, 0ull);
            for (int32_t k : *r.keys) {
                const unsigned long long v = (1ull << 32) | (uint32_t)k;
                uint32_t h = slot_hash_host((uint32_t)k) & (nsl - 1);
                while (dkeys[(size_t)(off + h)] != 0ull && dkeys[(size_t)(off + h)] != v) h = (h + 1) & (nsl - 1);
                dkeys[(size_t)(off + h)] = v;
            }
            dtabs.push_back(DkeyTab{f, off, nsl - 1});
        }
        F[f].iv0 = (int32_t)ivs.size();
        F[f].niv = (int32_t)r.niv;
        const size_t t0 = tiles.size();
        int64_t full = 0;
        for (int64_t i = 0; i < r.niv; ++i) full += probe_full_positions(r.iv[i].a, r.iv[i].b, fs.n, fs.B);
        const int64_t seg_len = probe_seg_len(full, fs.B);
        for (int64_t i = 0; i < r.niv; ++i) {
            const ProbeInterval& v = r.iv[i];
            ivs.push_back(ProbeIv{v.a, v.b, v.anchor, v.e_lo & 0xFFFFu, v.e_hi & 0xFFFFu, f, 0});
            probe_plan(v.a, v.b, fs.n, fs.B, (int32_t)(ivs.size() - 1), seg_len, &tiles, &segs);
        }
        probe_partials(&tiles, t0, fs.B, f, &ptiles);
        if (r.head) {  // anchors T(kB) of the blocks these tiles sit in
            for (size_t t = t0; t < tiles.size(); ++t) {
                const int64_t k = tiles[t].q0 / fs.B;
                if (!be.haw_ready[(size_t)k]) {
                    be.haw_ready[(size_t)k] = 1;
                    gw.push_back(GatherEnt{k * fs.B, f, 1});
                }
            }
        }
        preq.push_back(f);
        max_C = std::max(max_C, fs.C);
    };
    for (int32_t f : pend) {
        FileScan& fs = files[(size_t)f];
        Req& r = fs.req;
        switch (r.kind) {
            case Req::WEAK:
                gw_at[(size_t)f] = (int64_t)gw.size();
                for (int64_t i = 0; i < r.count; ++i) gw.push_back(GatherEnt{r.pos[i], f, 0});
                break;
            case Req::BYTES:
                gb_at[(size_t)f] = (int64_t)gb.size();
                for (int64_t i = 0; i < r.count; ++i) gb.push_back(GatherEnt{r.pos[i], f, 0});
                break;
            case Req::FLUSH:
                gw_at[(size_t)f] = (int64_t)gw.size();
                for (int64_t i = 0; i < r.count; ++i) gw.push_back(GatherEnt{r.pos[i], f, 0});
                gb_at[(size_t)f] = (int64_t)gb.size();
                for (int64_t i = 0; i < r.count2; ++i) gb.push_back(GatherEnt{r.pos2[i], f, 0});
                break;
            case Req::WAIT:
                break;
            case Req::WIN:
                win_at[(size_t)f] = win_bytes;
                copies.push_back(CopyEnt{fs.d_src + r.p, nullptr, r.w});  // dst fixed below
                win_bytes += pad16(r.w);
                max_win = std::max(max_win, r.w);
                break;
            case Req::FCHAIN:  // the chain's gathers (device memory), then its probe as PROBE
                fw_at[(size_t)f] = (int64_t)fw.size();
                for (int64_t i = 0; i < r.count; ++i) fw.push_back(GatherEnt{r.pos[i], f, 0});
                fb_at[(size_t)f] = (int64_t)fb.size();
                for (int64_t i = 0; i < r.count2; ++i) fb.push_back(GatherEnt{r.pos2[i], f, 0});
                fo_at[(size_t)f] = nfout;
                nfout += 2 * r.fchain.K;
                plan_probe(f);
                break;
            case Req::PROBE:
                plan_probe(f);
                break;
        }
    }
    // pinned staging of this round's inputs
    GatherEnt *hgw, *hgb;
    int32_t *how, *hreq;
    uint8_t *hob, *hwin;
    CopyEnt* hcp;
    ProbeIv* hiv;
    ProbeTile* ht;
    ProbeSeg* hsg;
    PartialTile* hpt;
    unsigned long long* hdk;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x) {
        if (x != hipSuccess && e == hipSuccess) e = x;
    };
    chk(pin(S->h_gw, (int64_t)gw.size(), &hgw));
    chk(pin(S->h_gb, (int64_t)gb.size(), &hgb));
    chk(pin(S->h_ow, (int64_t)gw.size(), &how));
    chk(pin(S->h_ob, (int64_t)gb.size(), &hob));
    chk(pin(S->h_win, win_bytes, &hwin));
    chk(pin(S->h_copies, (int64_t)copies.size(), &hcp));
    chk(pin(S->h_iv, (int64_t)ivs.size(), &hiv));
    chk(pin(S->h_tiles, (int64_t)tiles.size(), &ht));
    chk(pin(S->h_segs, (int64_t)segs.size(), &hsg));
    chk(pin(S->h_ptiles, (int64_t)ptiles.size(), &hpt));
    chk(pin(S->h_req, (int64_t)preq.size(), &hreq));
    chk(pin(S->h_dkeys, (int64_t)dkeys.size(), &hdk));
    CopyEnt* hrc = nullptr;
    chk(pin(S->h_rcp, 2, &hrc));
    GatherEnt* hfg = nullptr;
    FlushChainJob* hfj = nullptr;
    uint32_t* hfo = nullptr;
    int32_t nfj = 0;
    for (int32_t f : pend) nfj += files[(size_t)f].req.kind == Req::FCHAIN;
    if (nfj > 0) {
        chk(pin(S->h_fgw, (int64_t)(fw.size() + fb.size()), &hfg));
        chk(pin(S->h_fjobs, (int64_t)nfj, &hfj));
        chk(pin(S->h_fout, nfout, &hfo));
        chk(S->fc_dev.ensure(fw.size() * 4 + fb.size() + 16));
    }
    chk(S->partials.ensure((ptiles.size() + 1) * sizeof(int4)));
    chk(S->dslots.ensure((dkeys.size() + 1) * sizeof(unsigned long long)));
    if (e != hipSuccess) return e;
    if (!gw.empty()) memcpy(hgw, gw.data(), gw.size() * sizeof(GatherEnt));
    if (!gb.empty()) memcpy(hgb, gb.data(), gb.size() * sizeof(GatherEnt));
    for (size_t i = 0, k = 0; i < pend.size(); ++i) {
        const int32_t f = pend[i];
        if (win_at[(size_t)f] >= 0) {
            copies[k].dst = hwin + win_at[(size_t)f];
            ++k;
        }
    }
    if (!copies.empty()) memcpy(hcp, copies.data(), copies.size() * sizeof(CopyEnt));
    if (!ivs.empty()) memcpy(hiv, ivs.data(), ivs.size() * sizeof(ProbeIv));
    if (!tiles.empty()) memcpy(ht, tiles.data(), tiles.size() * sizeof(ProbeTile));
    if (!segs.empty()) memcpy(hsg, segs.data(), segs.size() * sizeof(ProbeSeg));
    if (!ptiles.empty()) memcpy(hpt, ptiles.data(), ptiles.size() * sizeof(PartialTile));
    if (!preq.empty()) memcpy(hreq, preq.data(), preq.size() * sizeof(int32_t));
    if (!dkeys.empty()) memcpy(hdk, dkeys.data(), dkeys.size() * sizeof(uint64_t));
    for (const DkeyTab& d : dtabs) {
        F[d.f].slots = S->dslots.as<unsigned long long>() + d.off;
        F[d.f].mask = d.mask;
    }

    // launches, one per kind, then one synchronisation
    if (!dkeys.empty())
        chk(hipMemcpyAsync(S->dslots.p, hdk, dkeys.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if (!preq.empty())
        chk(launch_probe_out_reset(S->first.as<ProbeOut>(), (uint32_t)files.size(), st));
    chk(launch_window_weak(F, hgw, (uint32_t)gw.size(), how, st));  // weak sums + head-mode anchors
    chk(launch_gather_bytes(F, hgb, (uint32_t)gb.size(), hob, st));
    chk(launch_copy_many(hcp, (uint32_t)copies.size(), max_win, st));
    // FCHAIN: the chains' sums and bytes, gathered into device memory for the chain kernel below
    int32_t* d_ftv = nullptr;
    uint8_t* d_fbv = nullptr;
    if (nfj > 0) {
        memcpy(hfg, fw.data(), fw.size() * sizeof(GatherEnt));
        memcpy(hfg + fw.size(), fb.data(), fb.size() * sizeof(GatherEnt));
        d_ftv = S->fc_dev.as<int32_t>();
        d_fbv = reinterpret_cast<uint8_t*>(d_ftv + fw.size());
        chk(launch_window_weak(F, hfg, (uint32_t)fw.size(), d_ftv, st));
        chk(launch_gather_bytes(F, hfg + fw.size(), (uint32_t)fb.size(), d_fbv, st));
    }
    if (!preq.empty()) {
        // The kernels read their descriptors where they are: pinned host memory, one PCIe round trip per workgroup,
        // which is nothing for a round's few tiles but the whole cost of a probe over a file's rest (a batched flush
        // chain of ~1600 intervals: ~30K tiles, 0.9 ms).  Above kProbeUpload tiles they go to device memory first.
        const ScanFile* dF = F;
        const ProbeIv* div = hiv;
        const ProbeTile* dt = ht;
        const PartialTile* dpt = hpt;
        const ProbeSeg* dsg = hsg;
        if (tiles.size() + segs.size() > kProbeUpload) {
            const size_t bf = pad16(files.size() * sizeof(ScanFile)), bi = pad16(ivs.size() * sizeof(ProbeIv)),
                         bt = pad16(tiles.size() * sizeof(ProbeTile)), bp = pad16(ptiles.size() * sizeof(PartialTile)),
                         bs = pad16(segs.size() * sizeof(ProbeSeg));
            chk(S->d_probe.ensure(bf + bi + bt + bp + bs + 16));
            if (e != hipSuccess) return e;
            uint8_t* d = S->d_probe.as<uint8_t>();
            chk(hipMemcpyAsync(d, F, files.size() * sizeof(ScanFile), hipMemcpyHostToDevice, st));
            chk(hipMemcpyAsync(d + bf, hiv, ivs.size() * sizeof(ProbeIv), hipMemcpyHostToDevice, st));
            chk(hipMemcpyAsync(d + bf + bi, ht, tiles.size() * sizeof(ProbeTile), hipMemcpyHostToDevice, st));
            if (!ptiles.empty())
                chk(hipMemcpyAsync(d + bf + bi + bt, hpt, ptiles.size() * sizeof(PartialTile), hipMemcpyHostToDevice, st));
            dF = reinterpret_cast<const ScanFile*>(d);
            div = reinterpret_cast<const ProbeIv*>(d + bf);
            dt = reinterpret_cast<const ProbeTile*>(d + bf + bi);
            dpt = reinterpret_cast<const PartialTile*>(d + bf + bi + bt);
            if (!segs.empty())
                chk(hipMemcpyAsync(d + bf + bi + bt + bp, hsg, segs.size() * sizeof(ProbeSeg), hipMemcpyHostToDevice, st));
            dsg = reinterpret_cast<const ProbeSeg*>(d + bf + bi + bt + bp);
        }
        if (nfj > 0) {  // every chain's desync into its intervals where the probe reads them, and to the host
            int32_t j = 0;
            for (int32_t f : pend) {
                const Req& r = files[(size_t)f].req;
                if (r.kind != Req::FCHAIN) continue;
                const FlushChain& q = r.fchain;
                hfj[j++] = FlushChainJob{d_ftv + fw_at[(size_t)f], d_fbv + fb_at[(size_t)f],
                                         const_cast<ProbeIv*>(div) + F[f].iv0 + r.npre, hfo + fo_at[(size_t)f], q.f, q.B,
                                         q.n, q.last, (int32_t)q.K, (int32_t)(r.niv - r.npre), q.el, q.eh};
            }
            chk(launch_flush_chain(hfj, (uint32_t)nfj, st));
        }
        ProbeArgs A;
        A.files = dF;
        A.ivs = div;
        A.tiles = dt;
        A.partials = S->partials.as<int4>();
        chk(launch_probe_first(A, (uint32_t)tiles.size(), dpt, (uint32_t)ptiles.size(), st));
        chk(launch_probe_long(A, dsg, (uint32_t)segs.size(), st));
        chk(launch_hit_window(F, hiv, hreq, (int32_t)preq.size(), max_C, st));
        // the answers into pinned memory by a copy kernel (capi.cpp copy_to_host: no copy-engine hand-off between
        // kernels, and every copy the profiler traces completes)
        hrc[0] = CopyEnt{S->first.as<uint8_t>(), S->h_first.as<uint8_t>(), (int64_t)(files.size() * sizeof(ProbeOut))};
        hrc[1] = CopyEnt{S->bucket.as<uint8_t>(), S->h_bucket.as<uint8_t>(),
                         (int64_t)(files.size() * HIT_BUCKET_INTS * sizeof(int32_t))};
        chk(launch_copy_many(hrc, 2, std::max(hrc[0].len, hrc[1].len), st));
    }
    chk(spin_sync(S, st));

    // answers
    const ProbeOut* hf = S->h_first.as<ProbeOut>();
    for (int32_t f : pend) {
        FileScan& fs = files[(size_t)f];
        Req& r = fs.req;
        switch (r.kind) {
            case Req::WEAK:
                for (int64_t i = 0; i < r.count; ++i) r.out_w[i] = e == hipSuccess ? how[gw_at[(size_t)f] + i] : 0;
                break;
            case Req::BYTES:
                for (int64_t i = 0; i < r.count; ++i) r.out_b[i] = e == hipSuccess ? hob[gb_at[(size_t)f] + i] : 0;
                break;
            case Req::FLUSH:
                for (int64_t i = 0; i < r.count; ++i) r.out_w[i] = e == hipSuccess ? how[gw_at[(size_t)f] + i] : 0;
                for (int64_t i = 0; i < r.count2; ++i) r.out_b2[i] = e == hipSuccess ? hob[gb_at[(size_t)f] + i] : 0;
                break;
            case Req::WAIT:
                break;
            case Req::WIN:
                r.win = hwin + win_at[(size_t)f];
                break;
            case Req::FCHAIN:
                for (int64_t i = 0; i < 2 * r.fchain.K; ++i) r.chain_out[i] = e == hipSuccess ? hfo[fo_at[(size_t)f] + i] : 0u;
                [[fallthrough]];
            case Req::PROBE:
                r.out = e == hipSuccess ? &hf[f] : nullptr;
                r.result = (e == hipSuccess && hf[f].first != ~0ull) ? (int64_t)hf[f].first : -1;
                break;
        }
    }
    return e;
}

hipError_t run_resolvers(rsh_ctx* c, BatchState* S, const std::shared_ptr<Batch>& bp, std::vector<FileScan>& files,
                         hipStream_t st, RoundCtl& ctl, int* rounds_out) {
    Batch& b = *bp;
    const int32_t NF = (int32_t)files.size();
    const bool trace = ctl.trace;
    const auto t0 = ctl.t0;
    bool& spec_launched = *ctl.spec_launched;
    int& spec_rc = *ctl.spec_rc;
    auto& launch_spec = ctl.launch_spec;
    const int defer_rounds = ctl.defer_rounds;
    const bool k1_launched = ctl.k1_launched;
    const int gen = ctl.gen;
    const int ncpu = WorkerCap::value() > 0 ? std::min(call_cores(), WorkerCap::value()) : call_cores();
    // spinning waiters: one core stays free for the coordinator
    const int32_t ncores = (spin_us() > 0 && ncpu > 2) ? ncpu - 1 : ncpu;
    // only the files still live get a worker: after the chain walks (or a leading speculation) most files are
    // done, and a worker per core spinning for one live file's rounds only eats the CPU quota
    std::vector<int32_t> live;
    for (int32_t f = 0; f < NF; ++f)
        if (!files[(size_t)f].done) live.push_back(f);
    const int32_t NL = (int32_t)live.size();
    const int32_t W = std::min<int32_t>({NL, ncores, kMaxWorkers});
    b.nworkers = W;
    b.worker_uc.resize((size_t)W);
    b.busy_ms.assign((size_t)W, 0.0);
    b.times.assign((size_t)W, HostTimes{});
    b.max_fiber_ms.assign((size_t)W, 0.0);
    for (int32_t i = 0; i < NL; ++i) files[(size_t)live[(size_t)i]].worker = i % W;
    // the fibers' stacks, kept across scans: a fresh 512 KiB allocation per file and scan is an mmap, page faults as
    // the fiber first runs, and a munmap, all on the resolvers' latency path (uninitialised: only touched pages commit)
    if (S->fiber_stacks.size() < (size_t)NL) S->fiber_stacks.resize((size_t)NL);
    std::vector<char*> stack_of((size_t)NL);
    for (int32_t i = 0; i < NL; ++i) {
        if (!S->fiber_stacks[(size_t)i]) S->fiber_stacks[(size_t)i].reset(new char[kFiberStack]);
        stack_of[(size_t)i] = S->fiber_stacks[(size_t)i].get();
    }
    char* const* stacks = stack_of.data();
    std::vector<std::thread> th;
    th.reserve((size_t)W);
    for (int32_t w = 0; w < W; ++w) {
        th.emplace_back([bp, &files, &live, w, NL, W, stacks] {
            Batch& b = *bp;
            uint64_t seen = 0;
            for (;;) {
                {
                    auto go = [&] { return b.gen.load(std::memory_order_acquire) != seen || b.quit.load(); };
                    spin_wait(go);
                    std::unique_lock<std::mutex> l(b.mu);
                    b.cv_work.wait(l, go);
                    if (b.quit) return;
                    seen = b.gen;
                }
                bool any = false;
                for (int32_t i = w; i < NL; i += W) {
                    FileScan& fs = files[(size_t)live[(size_t)i]];
                    if (fs.done) continue;
                    if (fs.pending && fs.req.kind == Req::WAIT && !b.landed.load(std::memory_order_acquire)) continue;
                    fs.pending = false;
                    if (!fs.started) {
                        fs.started = true;
                        fs.stack = stacks[i];
                        getcontext(&fs.uc);
                        fs.uc.uc_stack.ss_sp = fs.stack;
                        fs.uc.uc_stack.ss_size = kFiberStack;
                        fs.uc.uc_link = &b.worker_uc[(size_t)w];
                        const uintptr_t a = reinterpret_cast<uintptr_t>(&fs);
                        makecontext(&fs.uc, reinterpret_cast<void (*)()>(&fiber_main), 2, (uint32_t)(a >> 32),
                                    (uint32_t)a);
                    }
                    const auto tf = std::chrono::steady_clock::now();
                    swapcontext(&b.worker_uc[(size_t)w], &fs.uc);  // until its next request or its end
                    const double dt = ms_since(tf);
                    b.busy_ms[(size_t)w] += dt;
                    b.max_fiber_ms[(size_t)w] = std::max(b.max_fiber_ms[(size_t)w], dt);
                }
                // the worker stays while any file it owns is not done -- including files parked on WAIT, which
                // resume in a later round once the speculation lands (a worker whose live files all
                // waited used to leave for good, and the coordinator spun on their pending requests)
                for (int32_t i = w; i < NL && !any; i += W) any = !files[(size_t)live[(size_t)i]].done;
                std::lock_guard<std::mutex> l(b.mu);
                b.times[(size_t)w] = host_times();
                if (!any) {  // all of its files are done: leave (the coordinator's rounds no longer count it)
                    if (b.idle == --b.nworkers) b.cv_coord.notify_one();
                    return;
                }
                if (++b.idle == b.nworkers) b.cv_coord.notify_one();
            }
        });
    }
    {
        std::lock_guard<std::mutex> l(b.mu);
        b.gen = 1;
    }
    b.cv_work.notify_all();

    // coordinator: one round per "every live resolver is waiting or done"
    hipError_t err = hipSuccess;
    int rounds = 0;
    std::vector<int32_t> pend;
    auto t_round = std::chrono::steady_clock::now();
    for (;;) {
        {
            auto all_idle = [&] { return b.idle.load(std::memory_order_acquire) == b.nworkers; };
            spin_wait(all_idle);
            std::unique_lock<std::mutex> l(b.mu);
            b.cv_coord.wait(l, all_idle);
            pend.clear();
            for (int32_t f = 0; f < NF; ++f)
                if (!files[(size_t)f].done && files[(size_t)f].pending) pend.push_back(f);
            if (pend.empty()) {
                b.quit = true;
                break;
            }
        }
        ++rounds;
        if (!spec_launched && rounds > defer_rounds) {
            spec_rc = launch_spec();
            spec_launched = true;
        }
        if (spec_launched && spec_rc == RSH_OK && !b.landed.load() && hipEventQuery(c->ev_flags) == hipSuccess)
            b.landed.store(true, std::memory_order_release);
        if (spec_launched && spec_rc == RSH_OK && !b.aligned.load() && hipEventQuery(c->ev_spec) == hipSuccess)
            b.aligned.store(true, std::memory_order_release);
        if (k1_launched && !b.landed.load()) {  // stop the speculation of files resolved since it started
            for (int32_t f = 0; f < NF; ++f) {
                FileScan& fs = files[(size_t)f];
                if (fs.done && !fs.cancelled) {
                    fs.cancelled = true;
                    if (trace) fprintf(stderr, "[rsh-batch] round %3d  file %d resolved: its speculation stops\n", rounds, f);
                    const hipError_t ew = hipStreamWriteValue32(st, S->file_abort + f, (uint32_t)gen, 0);
                    if (ew != hipSuccess && err == hipSuccess) {  // a lost cancellation only costs time
                        err = ew;
                        note_error(ew, __LINE__, __FILE__);
                    }
                }
            }
        }
        const double wait_ms = ms_since(t_round);
        const auto t_serve = std::chrono::steady_clock::now();
        std::vector<int32_t> work;  // requests with device work; WAITs are answered by the landing alone
        for (int32_t f : pend)
            if (files[(size_t)f].req.kind != Req::WAIT) work.push_back(f);
        hipError_t e = hipSuccess;
        if (!work.empty()) {
            e = serve_round(c, S, files, work, c->stream);
        } else if (!b.landed.load()) {  // only waiting files: the speculation carries them
            e = spec_launched ? hipEventSynchronize(c->ev_flags) : hipErrorInvalidValue;
            if (e == hipSuccess) b.landed.store(true, std::memory_order_release);
            if (e == hipSuccess && hipEventQuery(c->ev_spec) == hipSuccess) b.aligned.store(true, std::memory_order_release);
            if (trace)
                fprintf(stderr, "[rsh-batch] round %3d  waited for the speculation: %.3f ms (landed at %.3f ms)\n", rounds,
                        ms_since(t_serve), ms_since(t0));
        }
        if (trace) {
            int kinds[7] = {0, 0, 0, 0, 0, 0, 0};
            for (int32_t f : pend) kinds[files[(size_t)f].req.kind]++;
            double bsum = 0, bmax = 0, fmax = 0;
            for (int32_t w = 0; w < W; ++w) {
                bsum += b.busy_ms[(size_t)w];
                bmax = std::max(bmax, b.busy_ms[(size_t)w]);
                fmax = std::max(fmax, b.max_fiber_ms[(size_t)w]);
            }
            fprintf(stderr, "[rsh-batch] round %3d  pending %3zu (weak %d bytes %d win %d probe %d flush %d chain %d)  wait "
                    "%.3f ms (host work: sum %.3f, max worker %.3f, max fiber %.3f)  serve %.3f ms%s  at %.3f ms\n",
                    rounds, pend.size(), kinds[0], kinds[1], kinds[2], kinds[3], kinds[5], kinds[6], wait_ms, bsum, bmax, fmax,
                    ms_since(t_serve), b.landed.load() ? "  [aligned]" : "", ms_since(t0));
            std::fill(b.busy_ms.begin(), b.busy_ms.end(), 0.0);
            std::fill(b.max_fiber_ms.begin(), b.max_fiber_ms.end(), 0.0);
        }
        t_round = std::chrono::steady_clock::now();
        if (e != hipSuccess && err == hipSuccess) {
            err = e;
            note_error(e, __LINE__, __FILE__);
        }
        {
            std::lock_guard<std::mutex> l(b.mu);
            b.idle = 0;
            ++b.gen;
        }
        b.cv_work.notify_all();
    }
    b.cv_work.notify_all();  // quit
    // every resolver is done and every worker idle: after quit a worker touches nothing but *bp
    for (std::thread& t : th) t.detach();
    *rounds_out = rounds;
    return err;
}

}  // namespace batch
}  // namespace rsh
