// capi.cpp -- the C-ABI of include/rsync_hip.h: contexts, device memory, the HIP scan backend and the
// host-side glue that mirrors Generator.sendItemizeAndChecksums / Sender.sendFiles per-file handling.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "device.h"
#include "host_md5.h"
#include "resolver.h"
#include "rsync_hip.h"

#include "ctx.h"
#include "options.h"
#include "rsync_hip_debug.h"

namespace {
// ------------------------------------------------------------------------------------------------
// HIP implementation of the resolver's services.
// ------------------------------------------------------------------------------------------------
constexpr size_t kFirstSlots = 1024;
// Device results to pinned host memory by a copy kernel (copy_few_kernel) rather than hipMemcpyAsync: between two
// kernels a D2H copy cost 47-100 us of idle queue (tools/queue_lat.hip case 8) where a kernel writing pinned memory
// cost none (case 9), and the profiler's async-copy tracing reported the copy engine's completions as never
// delivered.  The ranges travel in the kernel's arguments.
hipError_t copy_to_host(std::initializer_list<rsh::CopyEnt> ents, hipStream_t s) {
    rsh::CopyFew f{};
    for (const rsh::CopyEnt& x : ents)
        if (x.len > 0 && f.n < 4) f.e[f.n++] = x;
    return rsh::launch_copy_few(f, s);
}
constexpr int kScanWindows = 2;  // hit windows per probe in the single-file scan (hit_cache.h)
// Head mode launches the aligned speculation after scan_defer_steps (4) resolver steps or scan_defer_us (500 us;
// options.h) ...
constexpr int64_t kChainSteps = 2;  // ... after this many steps when the last event is a run of matches
// ... or at once when the first kLeadWindows (ctx.h) aligned source windows all carry chunk k's weak sum
// ... over the windows up to the last of scan_samples (256; 1024 until round 2: the same step time, r2_ab2)
// evenly spaced samples that still carries its chunk's sum
// windows one K1 launch digests in a single round of waves (2 waves/SIMD x 1024 SIMDs x 64 lanes): below this a
// launch over fewer windows is no faster
constexpr int64_t kRoundWindows = 131072;
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

class HipBackend : public rsh::ScanBackend {
  public:
    HipBackend(rsh_ctx* c, const uint8_t* d_src, int64_t n, rsh::ChunkTable& t, const int32_t* d_table_weak,
               const uint8_t seed[4])
        : rs_(c->stream), c_(c), x_(d_src), n_(n), t_(t), d_table_weak_(d_table_weak), B_(t.block_length),
          dl_(t.digest_length) {
        memcpy(seed_, seed, 4);
    }
    hipError_t err = hipSuccess;
    // the queue of the round trips (and of the tiled scan's loads): the context stream, or aux when the
    // speculation runs on the context stream (option scan_spec_queue, scan_device)
    hipStream_t rs_;
    int64_t na = 0;
    const int32_t* aw = nullptr;  // pinned host copies of the aligned speculation
    const uint8_t* as = nullptr;
    const uint8_t* fl = nullptr;
    rsh::ProbeTable table{};
    // Head mode: the speculation is still running on its own stream.  The resolver then sees no aligned
    // data, batched probes stay short, and the probe kernel's per-block anchors T(kB) come from c_->haw,
    // filled on demand for the blocks a probe touches.
    bool head = false;
    // the speculation covers windows [0, na) only (a prefix of the source's na_all): the probe's block anchors
    // beyond it come from c_->haw on demand, as in head mode
    bool partial = false;
    std::vector<uint8_t> haw_ready;
    std::function<void(uint8_t*)> md5_0;  // digest of window 0 (joins its host thread)

    int64_t aligned_count() override {  // the sums land after the flags (ev_spec after ev_flags)
        if (tiled) return aligned_end;
        if (head) return 0;
        if (!sums_ready) {
            if (lazy_na >= 0) {
                // scan_spec_queue: the first step that needs them downloads them (on rs_; the flags have landed) and
                // waits: the copy is tens of microseconds, the generic path's probe and host digest as long or longer
                CallTrace tr("sums_dl", lazy_na);
                ok(hipStreamWaitEvent(rs_, c_->ev_flags, 0));
                ok(copy_to_host({rsh::CopyEnt{c_->src_weak.as<uint8_t>(), c_->h_aw.as<uint8_t>(), lazy_na * 4},
                                                rsh::CopyEnt{c_->src_strong.as<uint8_t>(), c_->h_as.as<uint8_t>(),
                                                             dl_ > 0 ? lazy_na * dl_ : 0}},
                                rs_));
                ok(hipEventRecord(c_->ev_spec, rs_));
                ok(hipEventSynchronize(c_->ev_spec));
                lazy_na = -1;
            }
            sums_ready = err == hipSuccess && hipEventQuery(c_->ev_spec) == hipSuccess;
        }
        return sums_ready ? na : 0;
    }
    int64_t lazy_na = -1;  // >= 0: the speculation's sums (this many windows) are still on the device
    int64_t flags_count() override { return tiled ? aligned_end : head ? 0 : na; }
    bool sums_ready = false;
    int64_t max_batch() override { return head ? 4 : 4096; }
    int64_t max_batch_at(int64_t f) override {  // a batch's intervals, bytes and windows stay in the tile
        if (!tiled) return max_batch();
        ensure(f);
        const int64_t hi = std::min(n_, tile_lo + tile_T + tile_H);
        return std::max<int64_t>(1, std::min<int64_t>(max_batch(), (hi - f - B_ - 1) / (10 * B_)));
    }
    bool one_round(int64_t a, int64_t b) override { return !tiled || a / tile_T == b / tile_T; }

    // ---- tiled source (rsh_match_scan_tiled): HBM holds [tile_lo, tile_lo + tile_T + tile_H) of the
    // source, tile_T a multiple of B and tile_H >= 16 B.  Every device question starts at or after the
    // scan position, which only grows, and reaches at most 10 B + 1 past it (a flush interval and its
    // window); the batched flush chain is capped by max_batch_at.  So each question is answered from the
    // tile that holds its first position, and tiles only advance.  Loading a tile copies it in (fill) and
    // runs the aligned speculation over the windows that start in it. ----
    bool tiled = false;
    int64_t tile_T = 0, tile_H = 0, tile_lo = -1;
    uint8_t* tile_buf = nullptr;
    int64_t aligned_end = 0, tiles_loaded = 0;
    std::function<hipError_t(uint8_t* dst, int64_t off, int64_t len)> fill;  // synchronous
    const int32_t* d_table_strong = nullptr;
    void ensure(int64_t a) {
        if (!tiled || err != hipSuccess) return;
        if (tile_lo >= 0 && a >= tile_lo && (a < tile_lo + tile_T || tile_lo + tile_T >= n_)) return;
        load_tile(a / tile_T * tile_T);
    }
    void load_tile(int64_t lo) {
        CallTrace tr("tile_load", lo);
        if (ph_s0_ >= 0 && !ph_landed_) ok(hipEventSynchronize(c_->ev_phase[ph_set_]));  // it reads the old tile
        const int64_t hi = std::min(n_, lo + tile_T + tile_H);
        ok(fill(tile_buf, lo, hi - lo));
        if (err != hipSuccess) return;
        tile_lo = lo;
        x_ = tile_buf - lo;  // data[p] for p in [lo, hi)
        ++tiles_loaded;
        // the windows wholly inside the tile (the file's last window when the tile reaches the end)
        const int64_t na_all = (n_ + B_ - 1) / B_;
        const int64_t k0 = lo / B_, k1 = hi == n_ ? na_all : (hi - B_) / B_ + 1;
        const int64_t C = t_.chunk_count, f1 = std::min(k1, C);
        ok(rsh::launch_block_sums(x_ + k0 * B_, std::min(n_, k1 * B_) - k0 * B_, (uint32_t)B_, (uint32_t)(k1 - k0),
                                  (uint32_t)dl_, seed_word(seed_), c_->src_weak.as<int32_t>() + k0,
                                  c_->src_strong.as<uint8_t>() + k0 * dl_, rs_));
        if (f1 > k0)
            ok(rsh::launch_chain_flags(c_->src_weak.as<int32_t>() + k0, c_->src_strong.as<uint8_t>() + k0 * dl_,
                                       d_table_weak_ + k0, reinterpret_cast<const uint8_t*>(d_table_strong) + k0 * dl_,
                                       (uint32_t)(f1 - k0), (uint32_t)dl_, c_->flags.as<uint8_t>() + k0, rs_));
        ok(copy_to_host({rsh::CopyEnt{c_->src_weak.as<uint8_t>() + 4 * k0, c_->h_aw.as<uint8_t>() + 4 * k0, (k1 - k0) * 4},
                         rsh::CopyEnt{c_->src_strong.as<uint8_t>() + k0 * dl_, c_->h_as.as<uint8_t>() + k0 * dl_,
                                      (k1 - k0) * dl_},
                         rsh::CopyEnt{c_->flags.as<uint8_t>() + k0, c_->h_fl.as<uint8_t>() + k0, f1 - k0}},
                        rs_));
        ok(hipStreamSynchronize(rs_));
        bytes_read += std::min(n_, k1 * B_) - k0 * B_;
        aligned_end = k1;
    }
    const int32_t* aligned_weak() override { return aw; }
    const uint8_t* aligned_strong() override { return as; }
    const uint8_t* chain_flags() override { return fl; }

    void weak_many(const int64_t* pos, int64_t count, int32_t* out) override {
        if (count <= 0) return;
        if (count == 1 && pos[0] == t_pos_) {  // fetched with (or derived from) a probe result
            out[0] = t_val_;
            return;
        }
        CallTrace tr("weak_many", count);
        ensure(*std::min_element(pos, pos + count));
        bytes_read += count * B_;
        rsh::GatherEnt* hp = pin<rsh::GatherEnt>(c_->h_pos, count);
        int32_t* ho = pin<int32_t>(c_->h_out, count);
        rsh::ScanFile* F = file();
        if (err != hipSuccess) return;
        for (int64_t i = 0; i < count; ++i) hp[i] = rsh::GatherEnt{pos[i], 0, 0};
        ok(rsh::launch_window_weak(F, hp, (uint32_t)count, ho, rs_));
        ok(hipStreamSynchronize(rs_));
        memcpy(out, ho, (size_t)count * sizeof(int32_t));
    }
    void bytes_many(const int64_t* pos, int64_t count, uint8_t* out) override {
        if (count <= 0) return;
        CallTrace tr("bytes_many", count);
        ensure(*std::min_element(pos, pos + count));
        bytes_read += count;
        rsh::GatherEnt* hp = pin<rsh::GatherEnt>(c_->h_pos, count);
        uint8_t* ho = pin<uint8_t>(c_->h_out, count);
        rsh::ScanFile* F = file();
        if (err != hipSuccess) return;
        for (int64_t i = 0; i < count; ++i) hp[i] = rsh::GatherEnt{pos[i], 0, 0};
        ok(rsh::launch_gather_bytes(F, hp, (uint32_t)count, ho, rs_));
        ok(hipStreamSynchronize(rs_));
        memcpy(out, ho, (size_t)count);
    }
    void flush_gather(const int64_t* tpos, int64_t nt, int32_t* tv, const int64_t* bpos, int64_t nb,
                      uint8_t* bv) override {
        if (nt <= 0 || nb <= 0) {
            ScanBackend::flush_gather(tpos, nt, tv, bpos, nb, bv);
            return;
        }
        CallTrace tr("flush_gather", nt);
        ensure(std::min(*std::min_element(tpos, tpos + nt), *std::min_element(bpos, bpos + nb)));
        bytes_read += nt * B_ + nb;
        rsh::GatherEnt* hp = pin<rsh::GatherEnt>(c_->h_pos, nt + nb);
        int32_t* ho = pin<int32_t>(c_->h_out, nt + (nb + 3) / 4);
        rsh::ScanFile* F = file();
        if (err != hipSuccess) return;
        for (int64_t i = 0; i < nt; ++i) hp[i] = rsh::GatherEnt{tpos[i], 0, 0};
        for (int64_t i = 0; i < nb; ++i) hp[nt + i] = rsh::GatherEnt{bpos[i], 0, 0};
        uint8_t* hb = reinterpret_cast<uint8_t*>(ho + nt);
        ok(rsh::launch_window_weak(F, hp, (uint32_t)nt, ho, rs_));
        ok(rsh::launch_gather_bytes(F, hp + nt, (uint32_t)nb, hb, rs_));
        ok(hipStreamSynchronize(rs_));
        memcpy(tv, ho, (size_t)nt * sizeof(int32_t));
        memcpy(bv, hb, (size_t)nb);
    }
    // A single window's digest is one serial MD5 chain: 64-wide waves give it nothing, so the rare
    // resolver misses (first table hit after a reset) are digested on the host from a D2H copy.
    void md5_at(int64_t p, uint8_t out[16]) override {
        CallTrace tr("md5_at", p);
        const int64_t w = std::min<int64_t>(B_, n_ - p);
        if (p == 0 && md5_0) {  // computed on a host thread since the scan started
            md5_0(out);
            return;
        }
        int slot = -1;
        for (int k = 0; k < kScanWindows; ++k)
            if (p == win_pos_[k]) slot = k;
        if (slot > 0) {  // digested on a host thread since the probe returned
            if (win_md5_[slot].joinable()) win_md5_[slot].join();
            memcpy(out, win_digest_[slot], 16);
            return;
        }
        if (slot == 0) {  // the window came back with the probe result
            rsh::HostMd5 h;
            h.update(c_->h_hit.as<uint8_t>() + 16 + (int64_t)slot * B_, (size_t)w);
            h.update(seed_, 4);
            h.final(out);
            return;
        }
        ensure(p);
        uint8_t* hw = pin<uint8_t>(c_->h_win, w);
        if (err != hipSuccess) return;
        bytes_read += w;
        ok(rsh::launch_copy_to_host(x_ + p, w, hw, rs_));
        ok(hipStreamSynchronize(rs_));
        rsh::HostMd5 h;
        h.update(hw, (size_t)w);
        h.update(seed_, 4);
        h.final(out);
    }
    // The batched flush chain in one round trip: the gathers into device memory, the chain kernel writing the
    // chain's intervals' desync into the probe's interval list, then the probe (first_hit with fc_ set).
    int64_t flush_probe(const rsh::ProbeInterval* pre, int64_t npre, const rsh::FlushChain& q,
                        std::vector<rsh::FlushStep>* steps, std::vector<rsh::ProbeInterval>* ivs,
                        const std::vector<int32_t>* keys) override {
        rsh::flush_intervals(q, steps, ivs);
        if (ivs->empty()) return ScanBackend::flush_probe(pre, npre, q, steps, ivs, keys);
        std::vector<int64_t> tpos, bpos;
        rsh::flush_positions(q, &tpos, &bpos);
        std::vector<rsh::ProbeInterval> all(pre, pre + npre);
        all.insert(all.end(), ivs->begin(), ivs->end());
        std::vector<uint32_t> out((size_t)(2 * q.K));
        fc_ = Chain{&q, &tpos, &bpos, npre, out.data()};
        const int64_t p = first_hit(all.data(), (int64_t)all.size(), keys);
        fc_ = Chain{};
        for (size_t i = 0; i < steps->size(); ++i) {
            (*steps)[i].elo = out[2 * i];
            (*steps)[i].ehi = out[2 * i + 1];
            if (i < ivs->size()) {
                (*ivs)[i].e_lo = out[2 * i];
                (*ivs)[i].e_hi = out[2 * i + 1];
            }
        }
        return p;
    }
    struct Chain {  // flush_probe's chain, for the first_hit call it makes
        const rsh::FlushChain* q = nullptr;
        const std::vector<int64_t>* tpos = nullptr;
        const std::vector<int64_t>* bpos = nullptr;
        int64_t npre = 0;
        uint32_t* out = nullptr;
    } fc_;
    int64_t first_hit(const rsh::ProbeInterval* iv, int64_t count, const std::vector<int32_t>* keys) override {
        rsh::ProbeInterval one;
        if (count == 1 && !fc_.q) {  // answered by the previous probe's hit list, or cut to its unprobed part
            int64_t p = -1, a2 = iv[0].a;
            int32_t T = 0;
            if (cache_.lookup(iv[0], keys, &p, &T, &a2)) {
                if (p >= 0) {
                    t_pos_ = p;
                    t_val_ = T;
                }
                return p;
            }
            one = iv[0];
            one.a = a2;
            iv = &one;
        }
        CallTrace tr(fc_.q ? "flush_chain" : "first_hit", count);
        ensure(fc_.q ? std::min(iv[0].a, fc_.q->f) : iv[0].a);
        bytes_read += probe_bytes(iv, count, B_);
        if (fc_.q) bytes_read += (int64_t)fc_.tpos->size() * B_ + (int64_t)fc_.bpos->size();
        rsh::ProbeTable tab = table;
        if (keys) {
            const uint32_t ns = pow2_at_least(2 * keys->size() + 2);
            ok(c_->dslots.ensure(ns * sizeof(unsigned long long)));
            int32_t* hk = pin<int32_t>(c_->h_keys, (int64_t)keys->size() + 1);
            if (err != hipSuccess) return -1;
            if (!keys->empty()) memcpy(hk, keys->data(), keys->size() * sizeof(int32_t));
            ok(rsh::launch_table_clear(c_->dslots.as<unsigned long long>(), ns, rs_));
            ok(rsh::launch_table_insert(c_->dslots.as<unsigned long long>(), ns - 1, hk, (uint32_t)keys->size(),
                                        rs_));
            tab.slots = c_->dslots.as<unsigned long long>();
            tab.mask = ns - 1;
        }
        tiles_.clear();
        segs_.clear();
        ptiles_.clear();
        int64_t full = 0;
        for (int64_t i = 0; i < count; ++i) full += rsh::probe_full_positions(iv[i].a, iv[i].b, n_, B_);
        const int64_t seg_len = tiled ? 0 : rsh::probe_seg_len(full, B_);  // (tiled: one tile of the source in HBM)
        for (int64_t i = 0; i < count; ++i) rsh::probe_plan(iv[i].a, iv[i].b, n_, B_, (int32_t)i, seg_len, &tiles_, &segs_);
        rsh::probe_partials(&tiles_, 0, B_, 0, &ptiles_);
        rsh::ProbeIv* hiv = pin<rsh::ProbeIv>(c_->h_iv, count + 1);
        rsh::ProbeTile* ht = pin<rsh::ProbeTile>(c_->h_tiles, (int64_t)tiles_.size() + 1);
        rsh::PartialTile* hpt = pin<rsh::PartialTile>(c_->h_ptiles, (int64_t)ptiles_.size() + 1);
        rsh::ProbeSeg* hsg = pin<rsh::ProbeSeg>(c_->h_psegs, (int64_t)segs_.size() + 1);
        rsh::ProbeOut* hf = pin<rsh::ProbeOut>(c_->h_first, 1);
        join_window_digests();  // h_hit is about to be overwritten
        uint8_t* hh = pin<uint8_t>(c_->h_hit, 16 + kScanWindows * B_);
        int32_t* hb = pin<int32_t>(c_->h_bucket, rsh::HIT_BUCKET_INTS + 1);  // + the request list {0}
        rsh::ScanFile* F = file();
        ok(c_->partials.ensure((ptiles_.size() + 1) * sizeof(int4)));
        ok(c_->bucket.ensure(rsh::HIT_BUCKET_INTS * sizeof(int32_t)));
        // result records preset ("none") in batches: one reset launch per kFirstSlots probes
        ok(c_->first.ensure(kFirstSlots * sizeof(rsh::ProbeOut)));
        if (err != hipSuccess) return -1;
        if (c_->first_used % kFirstSlots == 0)
            ok(rsh::launch_probe_out_reset(c_->first.as<rsh::ProbeOut>(), (uint32_t)kFirstSlots, rs_));
        rsh::ProbeOut* d_first = c_->first.as<rsh::ProbeOut>() + c_->first_used++ % kFirstSlots;
        for (int64_t i = 0; i < count; ++i)
            hiv[i] = rsh::ProbeIv{iv[i].a, iv[i].b, iv[i].anchor, iv[i].e_lo & 0xFFFFu, iv[i].e_hi & 0xFFFFu, 0, 0};
        if (!tiles_.empty()) memcpy(ht, tiles_.data(), tiles_.size() * sizeof(rsh::ProbeTile));
        if (!ptiles_.empty()) memcpy(hpt, ptiles_.data(), ptiles_.size() * sizeof(rsh::PartialTile));
        if (!segs_.empty()) memcpy(hsg, segs_.data(), segs_.size() * sizeof(rsh::ProbeSeg));
        F->aligned_weak = (head || partial) ? c_->haw.as<int32_t>() : c_->src_weak.as<int32_t>();
        F->slots = tab.slots;
        F->mask = tab.mask;
        F->out = d_first;
        F->iv0 = 0;
        F->niv = (int32_t)count;
        F->bucket = c_->bucket.as<int32_t>();
        F->hit = hh;
        F->nwin = kScanWindows;
        if (head || partial) {  // anchors T(kB) for the blocks these tiles sit in
            anchors_.clear();
            for (const rsh::ProbeTile& t : tiles_) {
                const int64_t k = t.q0 / B_;
                if (!haw_ready[(size_t)k]) {
                    haw_ready[(size_t)k] = 1;
                    anchors_.push_back(rsh::GatherEnt{k * B_, 0, 1});
                }
            }
            if (!anchors_.empty()) {
                rsh::GatherEnt* hp = pin<rsh::GatherEnt>(c_->h_pos, (int64_t)anchors_.size());
                if (err != hipSuccess) return -1;
                memcpy(hp, anchors_.data(), anchors_.size() * sizeof(rsh::GatherEnt));
                ok(rsh::launch_window_weak(F, hp, (uint32_t)anchors_.size(), nullptr, rs_));
            }
        }
        uint32_t* hfo = nullptr;
        if (fc_.q) {  // the chain's gathers into device memory, then the chain into hiv[npre, count) and hfo
            const int64_t nt = (int64_t)fc_.tpos->size(), nb = (int64_t)fc_.bpos->size();
            rsh::GatherEnt* hfg = pin<rsh::GatherEnt>(c_->h_fgw, nt + nb);
            rsh::FlushChainJob* hj = pin<rsh::FlushChainJob>(c_->h_fjobs, 1);
            hfo = pin<uint32_t>(c_->h_fout, 2 * fc_.q->K);
            ok(c_->fc_dev.ensure((size_t)(nt * 4 + nb + 16)));
            if (err != hipSuccess) return -1;
            for (int64_t i = 0; i < nt; ++i) hfg[i] = rsh::GatherEnt{(*fc_.tpos)[(size_t)i], 0, 0};
            for (int64_t i = 0; i < nb; ++i) hfg[nt + i] = rsh::GatherEnt{(*fc_.bpos)[(size_t)i], 0, 0};
            int32_t* d_tv = c_->fc_dev.as<int32_t>();
            uint8_t* d_bv = reinterpret_cast<uint8_t*>(d_tv + nt);
            ok(rsh::launch_window_weak(F, hfg, (uint32_t)nt, d_tv, rs_));
            ok(rsh::launch_gather_bytes(F, hfg + nt, (uint32_t)nb, d_bv, rs_));
            const rsh::FlushChain& q = *fc_.q;
            *hj = rsh::FlushChainJob{d_tv, d_bv, hiv + fc_.npre, hfo, q.f, q.B, q.n, q.last, (int32_t)q.K,
                                     (int32_t)(count - fc_.npre), q.el, q.eh};
            ok(rsh::launch_flush_chain(hj, 1, rs_));
        }
        rsh::ProbeArgs A;
        A.files = F;
        A.ivs = hiv;
        A.tiles = ht;
        A.partials = c_->partials.as<int4>();
        ok(rsh::launch_probe_first(A, (uint32_t)tiles_.size(), hpt, (uint32_t)ptiles_.size(), rs_));
        ok(rsh::launch_probe_long(A, hsg, (uint32_t)segs_.size(), rs_));
        // the resolver's next questions at a hit are T(p), the bucket of the key that hit and (usually) the
        // MD5 of the window at p: answer them in this round trip
        int32_t* req = hb + rsh::HIT_BUCKET_INTS;
        *req = 0;
        ok(rsh::launch_hit_window(F, hiv, req, 1, t_.chunk_count, rs_));
        ok(copy_to_host(
                        {rsh::CopyEnt{reinterpret_cast<const uint8_t*>(d_first), reinterpret_cast<uint8_t*>(hf),
                                      (int64_t)sizeof(rsh::ProbeOut)},
                         rsh::CopyEnt{c_->bucket.as<uint8_t>(), reinterpret_cast<uint8_t*>(hb),
                                      (int64_t)(rsh::HIT_BUCKET_INTS * sizeof(int32_t))}},
                        rs_));
        ok(hipStreamSynchronize(rs_));
        if (fc_.q && err == hipSuccess) {  // the chain's desync: to the caller, and into the intervals the cache keeps
            memcpy(fc_.out, hfo, (size_t)(2 * fc_.q->K) * sizeof(uint32_t));
            rsh::ProbeInterval* civ = const_cast<rsh::ProbeInterval*>(iv);  // (flush_probe's own list)
            for (int64_t i = fc_.npre; i < count; ++i) {
                civ[i].e_lo = hfo[2 * (i - fc_.npre)];
                civ[i].e_hi = hfo[2 * (i - fc_.npre) + 1];
            }
        }
        if (count == 1) cache_.fill(iv[0], keys, *hf, n_ - B_);
        else cache_.fill_batch(iv, count, keys, *hf, n_ - B_);
        if (hf->first == ~0ull) return -1;
        rsh::window_slots(*hf, kScanWindows, win_pos_);
        for (int k = 1; k < kScanWindows; ++k)
            if (win_pos_[k] >= 0) {
                const int64_t wk = std::min<int64_t>(B_, n_ - win_pos_[k]);
                const uint8_t* src = hh + 16 + (int64_t)k * B_;
                win_md5_[k] = std::thread([this, k, wk, src] {
                    rsh::HostMd5 h;
                    for (int64_t o = 0; o < wk; o += kDigestPiece) {  // stops early once nobody can ask for it
                        if (win_cancel_.load(std::memory_order_relaxed)) return;
                        h.update(src + o, (size_t)std::min<int64_t>(kDigestPiece, wk - o));
                    }
                    h.update(seed_, 4);
                    h.final(win_digest_[k]);
                });
            }
        t_pos_ = (int64_t)hf->first;
        t_val_ = *reinterpret_cast<const int32_t*>(hh);
        prime_from_probe(t_, *hf, hb);
        return t_pos_;
    }

    // ---- phase-shifted speculation (resolver.h ScanBackend::phase_hint / phase_sums): K1 over [s0, n) with
    // the received header's B and dl, on the aux stream behind whatever runs there, one at a time ----
    int64_t ph_launches = 0;
    double phase_ms = 0;  // the K1s of the phase speculations that landed
    void phase_hint(int64_t s) override {
        if (ph_s0_ >= 0 && s >= ph_s0_ && (s - ph_s0_) % B_ == 0 && s < ph_s0_ + ph_count_ * B_) return;  // covered
        ensure(s);
        // windows wholly in the data the device holds: the rest of the file, or of the tile
        const int64_t hi = tiled ? std::min(n_, tile_lo + tile_T + tile_H) : n_;
        const int64_t count = hi == n_ ? (n_ - s + B_ - 1) / B_ : (hi - s - B_) / B_ + 1;
        if (count < kPhaseMinWindows || ph_launches >= kPhaseMaxLaunches || err != hipSuccess || !phase_on()) return;
        phase_stop();  // one at another phase is dead work now
        CallTrace tr("phase_spec", s);
        ph_gen_ = ++c_->gen;
        hipStream_t ps = c_->phase;  // its own stream: it does not queue behind a prefix speculation on aux
        // The launch this one replaces may still be draining on another stream (the segmented launch on aux
        // keeps its prefix waves and tail lanes running after the phase word stops its phase waves) and
        // still write its sums and their host copies: this launch takes the other buffer set, after that
        // set's previous launch and downloads.
        const int set = 1 - c_->ph_set;
        ok(hipStreamWaitEvent(ps, c_->ev_in, 0));
        ok(hipStreamWaitEvent(ps, c_->ev_phase[set], 0));
        ok(hipEventRecord(c_->ev_pha[set], ps));
        ok(rsh::launch_block_sums(x_ + s, std::min(n_ - s, count * B_), (uint32_t)B_, (uint32_t)count, (uint32_t)dl_,
                                  seed_word(seed_),
                                  c_->ph_weak[set].as<int32_t>(), c_->ph_strong[set].as<uint8_t>(), ps,
                                  c_->abort_word + rsh_ctx::kPhaseWord, ph_gen_));
        ok(hipEventRecord(c_->ev_phb[set], ps));
        ok(copy_to_host({rsh::CopyEnt{c_->ph_weak[set].as<uint8_t>(), c_->h_pw[set].as<uint8_t>(), count * 4},
                         rsh::CopyEnt{c_->ph_strong[set].as<uint8_t>(), c_->h_ps[set].as<uint8_t>(), count * dl_}},
                        ps));
        ok(hipEventRecord(c_->ev_phase[set], ps));
        c_->ph_set = set;
        ph_set_ = set;
        if (err != hipSuccess) return;
        ph_s0_ = s;
        ph_count_ = count;
        ph_landed_ = false;
        ++ph_launches;
    }
    bool phase_sums(int64_t s, bool wait, rsh::PhaseView* v) override {
        if (ph_s0_ < 0 || s < ph_s0_ || (s - ph_s0_) % B_ != 0 || s >= ph_s0_ + ph_count_ * B_ || err != hipSuccess)
            return false;
        if (!ph_landed_) {
            // a phase K1 that has finished leaves only its sums' download (~1 MB): waiting for it beats a host
            // digest of the window (0.13 ms at B = 128 KiB), the resolver's alternative at a hit
            if (wait || hipEventQuery(c_->ev_phb[ph_set_]) == hipSuccess) {
                CallTrace tr("phase_wait", s);
                ok(hipEventSynchronize(c_->ev_phase[ph_set_]));
                ph_landed_ = err == hipSuccess;
            } else {
                ph_landed_ = hipEventQuery(c_->ev_phase[ph_set_]) == hipSuccess;
            }
            if (!ph_landed_) return false;
            bytes_read += std::min(n_ - ph_s0_, ph_count_ * B_);
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, c_->ev_pha[ph_set_], c_->ev_phb[ph_set_]) == hipSuccess) phase_ms += ms;
        }
        v->s0 = ph_s0_;
        v->count = ph_count_;
        v->w = c_->h_pw[ph_set_].as<int32_t>();
        v->st = c_->h_ps[ph_set_].as<uint8_t>();
        return true;
    }
    // A phase-shifted speculation the caller launched (the segmented prefix + phase launch, scan_device) over
    // windows s0 + kB, k < count, generation gen, into buffer set `set`, landing on ev_phase[set]: from now on
    // this backend's.
    void phase_adopt(int64_t s0, int64_t count, int gen, int set) {
        ph_set_ = set;
        ph_s0_ = s0;
        ph_count_ = count;
        ph_gen_ = gen;
        ph_landed_ = false;
        ++ph_launches;
    }
    // A phase speculation still running when the scan ends (or moves to another phase) is stopped; later
    // work on the context stream waits until its waves have left.
    void phase_stop() {
        if (ph_s0_ >= 0 && !ph_landed_ && hipEventQuery(c_->ev_phase[ph_set_]) == hipErrorNotReady) {
            ok(hipStreamWriteValue32(rs_, c_->abort_word + rsh_ctx::kPhaseWord, (uint32_t)ph_gen_, 0));
            ok(hipStreamWaitEvent(rs_, c_->ev_phase[ph_set_], 0));
            // the caller's later work on the context stream (it may rewrite the source) after the draining waves
            if (rs_ != c_->stream) ok(hipStreamWaitEvent(c_->stream, c_->ev_phase[ph_set_], 0));
        }
        ph_s0_ = -1;
        ph_landed_ = false;
    }
    static bool phase_on() { return rsh::opt(rsh::OPT_SCAN_PHASE) != 0; }  // A/B: 0 = no phase speculation

  private:
    static constexpr int64_t kPhaseMinWindows = 8;    // shorter remainders resolve faster on the generic path
    static constexpr int64_t kPhaseMaxLaunches = 64;  // each covers the rest of the file
    int64_t ph_s0_ = -1, ph_count_ = 0;
    int ph_gen_ = 0;
    int ph_set_ = 0;  // the buffer set (rsh_ctx::ph_weak[i] ...) of the current phase launch
    bool ph_landed_ = false;

    template <class T>
    T* pin(PinnedBuf& b, int64_t count, int line = __builtin_LINE()) {
        ok(b.ensure((size_t)std::max<int64_t>(count, 1) * sizeof(T)), line);
        return b.as<T>();
    }
    void ok(hipError_t e, int line = __builtin_LINE()) {
        if (e != hipSuccess && err == hipSuccess) {
            err = e;
            note_error(e, line);
        }
    }
    rsh_ctx* c_;
    const uint8_t* x_;
    int64_t n_;
    rsh::ChunkTable& t_;
    const int32_t* d_table_weak_;  // the received table's weak sums on the device
    int64_t B_;
    int dl_;
    uint8_t seed_[4];
    std::vector<rsh::ProbeTile> tiles_;
    std::vector<rsh::PartialTile> ptiles_;
    std::vector<rsh::ProbeSeg> segs_;
    std::vector<rsh::GatherEnt> anchors_;
    // the scan as a batch of one file for the probe / gather kernels (pinned, device-readable)
    rsh::ScanFile* file() {
        rsh::ScanFile* F = pin<rsh::ScanFile>(c_->h_files, 1);
        if (err != hipSuccess) return F;
        F->data = x_;
        F->n = n_;
        F->B = (uint32_t)B_;
        F->aligned_weak = (head || partial) ? c_->haw.as<int32_t>() : c_->src_weak.as<int32_t>();
        F->table_weak = d_table_weak_;
        F->C = t_.chunk_count;
        F->nsmall = 0;  // key sets as probe hashes (tab.slots)
        return F;
    }
    int64_t win_pos_[rsh::HIT_WINDOWS] = {-1, -1, -1, -1};  // windows of the last probe's hits on the host (h_hit)
    // digests of the windows in slots 1 .. kScanWindows-1, started on host threads when the probe returns
    // (the resolver handles the first hit meanwhile); joined before the next probe overwrites h_hit
    std::thread win_md5_[rsh::HIT_WINDOWS];
    uint8_t win_digest_[rsh::HIT_WINDOWS][16];
    // set when the scan ends: a window digest still running then is never read (the join at the end of the
    // scan took ~0.09 ms for one 128 KiB window digested after the scan's last probe)
    std::atomic<bool> win_cancel_{false};
    static constexpr int64_t kDigestPiece = 8192;
    void join_window_digests() {
        for (std::thread& t : win_md5_)
            if (t.joinable()) t.join();
    }

  public:
    ~HipBackend() {
        win_cancel_.store(true, std::memory_order_relaxed);
        join_window_digests();
    }

  private:
    int64_t t_pos_ = -1;    // position of the last hit returned: its weak sum t_val_ is known
    int32_t t_val_ = 0;
    HitCache cache_;
};

}  // namespace

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
            ok(hipStreamSynchronize(st));
        }
    }
    ok(hipStreamSynchronize(c->stream));
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
    int gen = ++c->gen;  // a stopped speculation's generation; a later launch takes a new one
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
            flags_gen = ++c->stamp_seq;
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
        const int prep_gen = ++c->stamp_seq;
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
        {
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
    uint8_t md5_0[16];
    std::thread md5_0_thread([&] {
        rsh::HostMd5 hm;
        hm.update(c->h_win0.as<uint8_t>(), (size_t)w0);
        hm.update(seed, 4);
        hm.final(md5_0);
    });
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
            RSH_HIP(hipStreamWriteValue32(rs, c->abort_word, (uint32_t)gen, 0));
            gen = ++c->gen;
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
    if (on_ctx) {  // (aux) the table and the probe hash, after a tentative launch's abort (above)
        int rc;
        {
            CallTrace tr("table_work", C);
            rc = table_work();
        }
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
    // The prefix end (below) needs the weak sums of the aligned windows between the run's last matching sample
    // and the first that does not: launched now, ahead of the guess's first probe, so that they land in its
    // round trip instead of one of their own
    const int64_t pe_lo = run_last + 1, pe_hi = std::min<int64_t>(run_miss, nf - 1), pe_cnt = pe_hi - pe_lo + 1;
    int32_t* pe_w = nullptr;
    if (defer_prefix && guess_on && seg_on && run_miss > 0 && pe_cnt > 0 && pe_cnt <= 4096 && be.err == hipSuccess) {
        const size_t ents_at = ((size_t)pe_cnt * 4 + 63) & ~(size_t)63;
        RSH_HIP(c->h_pend.ensure(ents_at + (size_t)pe_cnt * sizeof(rsh::GatherEnt)));
        pe_w = c->h_pend.as<int32_t>();
        auto* pents = reinterpret_cast<rsh::GatherEnt*>(c->h_pend.as<uint8_t>() + ents_at);
        for (int64_t i = 0; i < pe_cnt; ++i) pents[i] = rsh::GatherEnt{(pe_lo + i) * B, 0, 0};
        auto* lf = reinterpret_cast<rsh::ScanFile*>(reinterpret_cast<rsh::GatherEnt*>(c->h_lead.as<uint8_t>() + lead_ents_at) +
                                                    nsamp + 1);
        RSH_HIP(rsh::launch_window_weak(lf, pents, (uint32_t)pe_cnt, pe_w, rs));
        be.bytes_read += pe_cnt * B;
    }
    if (guess_on && run_miss > 0 && (spec_launched || defer_prefix) && HipBackend::phase_on() && C >= 4) {
        CallTrace tr("phase_guess", run_miss);
        int64_t a = run_miss * B;
        const int64_t b = std::min<int64_t>(run_miss * B + 2 * B, n - 4 * B + 1);  // the edit may sit in window m
        for (int tries = 0; tries < 8 && a < b && be.err == hipSuccess; ++tries) {
            const rsh::ProbeInterval iv{a, b, a, 0, 0};
            const int64_t p = be.first_hit(&iv, 1, nullptr);
            if (p < 0) break;
            const int64_t pos[4] = {p, p + B, p + 2 * B, p + 3 * B};
            int32_t w[4];
            be.weak_many(pos, 4, w);
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
                const int gph = ++c->gen;
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
                    RSH_HIP(hipMemcpyAsync(c->segs.p, c->h_segs.p, bytes, hipMemcpyHostToDevice, ss));
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

extern "C" {

int rsh_abi_version(void) { return RSH_ABI_VERSION; }

const char* rsh_last_error(void) { return g_last_err; }

const char* rsh_strerror(int status) {
    switch (status) {
        case RSH_OK: return "ok";
        case RSH_E_INVAL: return "invalid argument";
        case RSH_E_PROTOCOL: return "checksum header rejected (RsyncProtocolException)";
        case RSH_E_OVERFLOW: return "chunk count is negative or greater than int max (ChunkOverflow)";
        case RSH_E_NOSPACE: return "event buffer too small";
        case RSH_E_DEVICE: return "HIP device error or no gfx950 device";
        case RSH_E_NOMEM: return "out of memory";
        case RSH_E_BUSY: return "context in use by another thread";
        case RSH_E_NOTFOUND: return "file not found (FileViewNotFound)";
        case RSH_E_OPEN: return "file cannot be opened (FileViewOpenFailed)";
        default: return "unknown status";
    }
}

int rsh_device_count(int* count) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (count) *count = c;
    return c > 0 ? RSH_OK : RSH_E_DEVICE;
}

int rsh_ctx_create(int device, rsh_ctx** out) {
    if (!out) return RSH_E_INVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return RSH_E_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RSH_E_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RSH_E_DEVICE;  // kernels are built for gfx950 only
    RSH_HIP(hipSetDevice(device));
    rsh_ctx* c = new (std::nothrow) rsh_ctx();
    if (!c) return RSH_E_NOMEM;
    c->device = device;
    c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->abort_word = nullptr;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->phase, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tab, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_spec, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_phase[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_phase[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_flags, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_prep, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->ev_k1a) != hipSuccess || hipEventCreate(&c->ev_k1b) != hipSuccess ||
        hipEventCreate(&c->ev_gen_a) != hipSuccess || hipEventCreate(&c->ev_gen_b) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rs_tail, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->ev_pha[0]) != hipSuccess || hipEventCreate(&c->ev_phb[0]) != hipSuccess ||
        hipEventCreate(&c->ev_pha[1]) != hipSuccess || hipEventCreate(&c->ev_phb[1]) != hipSuccess ||
        hipExtMallocWithFlags(reinterpret_cast<void**>(&c->abort_word), 256, hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(c->abort_word, 0, 256) != hipSuccess ||  // generations start at 1
        // recorded once, so that a launch may always wait for its buffer set's previous launch
        hipEventRecord(c->ev_phase[0], c->stream) != hipSuccess || hipEventRecord(c->ev_phase[1], c->stream) != hipSuccess) {
        delete c;
        return RSH_E_DEVICE;
    }
    if (ctx_warm(c) != hipSuccess) {
        (void)hipStreamSynchronize(c->stream);
        delete c;
        return RSH_E_DEVICE;
    }
    *out = c;
    return RSH_OK;
}

void rsh_ctx_destroy(rsh_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (hipStream_t st : {ctx->stream, ctx->aux, ctx->phase})  // nothing may still read or write its buffers
        if (st) (void)hipStreamSynchronize(st);
    delete ctx;
}

void* rsh_ctx_stream(rsh_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int rsh_ctx_sync(rsh_ctx* ctx) {
    if (!ctx) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->aux));    // includes a cancelled speculation draining
    RSH_HIP(hipStreamSynchronize(ctx->phase));  // a stopped phase-shifted speculation and its downloads
    return RSH_OK;
}

// The pass-sized buffers back to the device and host allocators (a Generator and a Sender context on one
// GPU each kept 2 x segment_bytes of HBM between segments).  Small round-trip buffers stay: they are what the next
// call would otherwise allocate on its latency path.
int rsh_ctx_trim(rsh_ctx* ctx) {
    if (!ctx) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    for (hipStream_t st : {ctx->stream, ctx->aux, ctx->phase}) RSH_HIP(hipStreamSynchronize(st));
    for (DevBuf* b : {&ctx->data, &ctx->weak, &ctx->strong, &ctx->seg_data, &ctx->seg_tab, &ctx->rcv[0], &ctx->rcv[1],
                      &ctx->rcv_ops[0], &ctx->rcv_ops[1], &ctx->out})
        b->release();
    for (PinnedBuf* b : {&ctx->h_stage, &ctx->h_rcv_ops[0], &ctx->h_rcv_ops[1], &ctx->h_out})
        b->release();
    if (ctx->h_win.cap > (1u << 20)) ctx->h_win.release();  // (a Receiver pass's pieces; the scan's windows are small)
    if (ctx->batch) {  // the batched scan's tables, hit map and fiber stacks (rebuilt on the next batched call)
        rsh::destroy_batch_state(ctx->batch);
        ctx->batch = nullptr;
    }
    return RSH_OK;
}

// Generator.getBlockLengthFor / pow2SquareRoot (Generator.java:198-206, 219-236).
int32_t rsh_block_length_for(int64_t file_size) {
    if (file_size <= 0) return 0;
    const int exponent = 63 - __builtin_clzll((unsigned long long)file_size);
    const int32_t bl = (int32_t)(1u << (exponent / 2));
    return bl > 512 ? bl : 512;  // MIN_BLOCK_SIZE (:186)
}

// Generator.getDigestLength (:208-212) with Util.log2 = Math.log(n) / Math.log(2) (Util.java:128-130),
// then max(minDigestLength, ...) (:873).
int32_t rsh_digest_length_for(int64_t file_size, int32_t block_length, int32_t min_digest_length) {
    if (file_size <= 0) return 0;  // Generator.java:873: digestLength 0 for an empty file
    const int64_t lf = (int64_t)(__builtin_log((double)file_size) / __builtin_log(2.0));
    const int64_t lb = (int64_t)(__builtin_log((double)block_length) / __builtin_log(2.0));
    int32_t r = ((int32_t)(10 + 2 * lf - lb) - 24) / 8;
    r = std::min(r, 16);
    r = std::max(r, 2);
    return std::max(r, min_digest_length);
}

int rsh_header_make(int32_t block_length, int32_t digest_length, int64_t file_size, rsh_header* out) {
    if (!out || block_length < 0 || file_size < 0) return RSH_E_INVAL;
    if (block_length == 0) {
        *out = rsh_header{0, 0, 0, 0};
        return RSH_OK;
    }
    const int64_t rem = file_size % block_length;
    const int64_t cc = file_size / block_length + (rem > 0 ? 1 : 0);
    if (cc > 2147483647LL) return RSH_E_OVERFLOW;
    *out = rsh_header{(int32_t)cc, block_length, digest_length, (int32_t)rem};
    return RSH_OK;
}

// Checksum.Header 4-arg ctor (Checksum.java:75-92); IllegalArgumentException -> RsyncProtocolException
// in Connection.receiveChecksumHeader (Connection.java:28-38).
int rsh_header_validate(const rsh_header* h) {
    if (!h) return RSH_E_INVAL;
    if (h->chunk_count < 0) return RSH_E_PROTOCOL;
    if (h->block_length == 0 && h->chunk_count > 0) return RSH_E_PROTOCOL;
    if (h->block_length < 0 || h->block_length > kMaxBlockLength) return RSH_E_PROTOCOL;
    if (h->remainder < 0 || h->remainder > h->block_length) return RSH_E_PROTOCOL;
    if (h->digest_length < 0) return RSH_E_PROTOCOL;
    return RSH_OK;
}

int rsh_block_sums_device(rsh_ctx* ctx, const void* d_data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                          void* d_weak, void* d_strong) {
    if (!ctx || !seed) return RSH_E_INVAL;
    const int rc = check_generator_header(n, h);
    if (rc != RSH_OK) return rc;
    if (h->chunk_count == 0) return RSH_OK;
    if (!d_data || !d_weak || (!d_strong && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    // the K1's own start / stop timestamps (rsh_debug_kernel_ms; no marker packets around it; option time_gen)
    if (rsh::opt(rsh::OPT_TIME_GEN) != 0) rsh::k1_timing_next(ctx->ev_gen_a, ctx->ev_gen_b);
    const hipError_t e = rsh::launch_block_sums(static_cast<const uint8_t*>(d_data), n, (uint32_t)h->block_length,
                                                (uint32_t)h->chunk_count, (uint32_t)h->digest_length, seed_word(seed),
                                                static_cast<int32_t*>(d_weak), static_cast<uint8_t*>(d_strong),
                                                ctx->stream);
    ctx->gen_timed = rsh::k1_timing_taken();
    rsh::k1_timing_next(nullptr, nullptr);
    RSH_HIP(e);
    return RSH_OK;
}

int rsh_block_sums(rsh_ctx* ctx, const uint8_t* data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                   int32_t* weak_out, uint8_t* strong_out) {
    if (!ctx || !seed) return RSH_E_INVAL;
    const int rc = check_generator_header(n, h);
    if (rc != RSH_OK) return rc;
    if (h->chunk_count == 0) return RSH_OK;
    if (!data || !weak_out || (!strong_out && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
    RSH_HIP(ctx->data.ensure((size_t)n));
    RSH_HIP(ctx->weak.ensure(C * 4));
    RSH_HIP(ctx->strong.ensure(C * dl + 1));
    RSH_HIP(hipMemcpyAsync(ctx->data.p, data, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    const int r2 = rsh_block_sums_device(ctx, ctx->data.p, n, h, seed, ctx->weak.p, ctx->strong.p);
    if (r2 != RSH_OK) return r2;
    RSH_HIP(hipMemcpyAsync(weak_out, ctx->weak.p, C * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (dl) RSH_HIP(hipMemcpyAsync(strong_out, ctx->strong.p, C * dl, hipMemcpyDeviceToHost, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_match_scan_device(rsh_ctx* ctx, const void* d_src, int64_t n, const rsh_header* h, const void* d_weak,
                          const void* d_strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap,
                          int64_t* n_ev, int64_t* literal, int64_t* matched, rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || n < 0) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    rsh::ResolveResult r;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        if (!d_src || (h->chunk_count > 0 && (!d_weak || (!d_strong && h->digest_length > 0)))) return RSH_E_INVAL;
        CallTrace tr("scan_call", n);  // with scan_device's teardown
        const int rc = scan_device(ctx, static_cast<const uint8_t*>(d_src), n, h, static_cast<const int32_t*>(d_weak),
                                   static_cast<const uint8_t*>(d_strong), nullptr, nullptr, seed, &r);
        if (rc != RSH_OK) return rc;
    }
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_match_scan(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                   const uint8_t* strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap, int64_t* n_ev,
                   uint8_t file_md5[16], int64_t* literal, int64_t* matched, rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || !file_md5 || n < 0 || (n > 0 && !src)) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    // the whole-file digest (Sender.java:1241,1326) is one serial chain: host thread, beside the device
    std::thread md5_thread([&] {
        rsh::HostMd5 m;
        if (n > 0) m.update(src, (size_t)n);
        m.final(file_md5);
    });
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
        if (C > 0 && (!weak || (!strong && dl > 0))) rc = RSH_E_INVAL;
        if (rc == RSH_OK && (ctx->data.ensure((size_t)n) != hipSuccess || ctx->weak.ensure(C * 4 + 4) != hipSuccess ||
                             ctx->strong.ensure(C * dl + 1) != hipSuccess))
            rc = RSH_E_NOMEM;
        if (rc == RSH_OK) {
            bool okc = hipMemcpyAsync(ctx->data.p, src, (size_t)n, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C) okc = okc && hipMemcpyAsync(ctx->weak.p, weak, C * 4, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C && dl)
                okc = okc && hipMemcpyAsync(ctx->strong.p, strong, C * dl, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            rc = okc ? scan_device(ctx, ctx->data.as<uint8_t>(), n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(),
                                   weak, strong, seed, &r)
                     : RSH_E_DEVICE;
        }
    }
    md5_thread.join();
    if (rc != RSH_OK) return rc;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_match_scan_tiled(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                         const uint8_t* strong, const uint8_t seed[4], int64_t tile_bytes, rsh_event* ev,
                         int64_t ev_cap, int64_t* n_ev, uint8_t file_md5[16], int64_t* literal, int64_t* matched,
                         rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || n < 0 || tile_bytes < 0 || (n > 0 && !src)) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    std::thread md5_thread;
    if (file_md5)
        md5_thread = std::thread([&] {
            rsh::HostMd5 m;
            if (n > 0) m.update(src, (size_t)n);
            m.final(file_md5);
        });
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
        if (C > 0 && (!weak || (!strong && dl > 0))) rc = RSH_E_INVAL;
        if (rc == RSH_OK && (ctx->weak.ensure(C * 4 + 4) != hipSuccess || ctx->strong.ensure(C * dl + 1) != hipSuccess))
            rc = RSH_E_NOMEM;
        if (rc == RSH_OK) {
            bool okc = true;
            if (C) okc = hipMemcpyAsync(ctx->weak.p, weak, C * 4, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C && dl)
                okc = okc && hipMemcpyAsync(ctx->strong.p, strong, C * dl, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            auto fill = [&](uint8_t* dst, int64_t off, int64_t len) -> hipError_t {
                const hipError_t e = hipMemcpyAsync(dst, src + off, (size_t)len, hipMemcpyHostToDevice, ctx->stream);
                return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
            };
            const int64_t tb = tile_bytes > 0 ? tile_bytes : kDefaultTile;
            rc = okc ? scan_tiled(ctx, fill, n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(), weak, strong, seed,
                                  tb, &r)
                     : RSH_E_DEVICE;
        }
    }
    if (md5_thread.joinable()) md5_thread.join();
    if (rc != RSH_OK) return rc;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_fetch_events(rsh_ctx* ctx, rsh_event* ev, int64_t ev_cap, int64_t* n_ev) {
    if (!ctx || !n_ev) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    *n_ev = (int64_t)ctx->last_ev.size();
    if (*n_ev > ev_cap || (!ev && *n_ev > 0)) return RSH_E_NOSPACE;
    if (*n_ev > 0) memcpy(ev, ctx->last_ev.data(), ctx->last_ev.size() * sizeof(rsh_event));
    return RSH_OK;
}

int rsh_file_md5(const uint8_t* data, int64_t n, uint8_t out[16]) {
    if (!out || n < 0 || (n > 0 && !data)) return RSH_E_INVAL;
    rsh::HostMd5 m;
    if (n > 0) m.update(data, (size_t)n);
    m.final(out);
    return RSH_OK;
}

int64_t rsh_tokens_size(const rsh_event* ev, int64_t n_ev) {
    int64_t size = 4 + 16;  // putInt(0) + file MD5
    for (int64_t i = 0; i < n_ev; ++i) {
        if (ev[i].kind == RSH_EV_LITERAL) size += ev[i].length + 4 * ((ev[i].length + kChunkSize - 1) / kChunkSize);
        else size += 4 * (int64_t)ev[i].count;
    }
    return size;
}

static inline uint8_t* put_int(uint8_t* o, int32_t v) {  // BufferedOutputChannel is little-endian (:50)
    for (int i = 0; i < 4; ++i) o[i] = (uint8_t)((uint32_t)v >> (8 * i));
    return o + 4;
}

int rsh_tokens_write(const uint8_t* src, const rsh_event* ev, int64_t n_ev, const uint8_t file_md5[16], uint8_t* out,
                     int64_t cap) {
    if (!out || !file_md5 || (n_ev > 0 && !ev)) return RSH_E_INVAL;
    if (rsh_tokens_size(ev, n_ev) > cap) return RSH_E_NOSPACE;
    uint8_t* o = out;
    for (int64_t i = 0; i < n_ev; ++i) {
        if (ev[i].kind == RSH_EV_LITERAL) {  // Sender.sendDataFrom (:794-809)
            if (!src) return RSH_E_INVAL;
            for (int64_t cur = ev[i].offset, end = ev[i].offset + ev[i].length; cur < end;) {
                const int64_t len = std::min<int64_t>(kChunkSize, end - cur);
                o = put_int(o, (int32_t)len);
                memcpy(o, src + cur, (size_t)len);
                o += len;
                cur += len;
            }
        } else {
            for (int32_t j = 0; j < ev[i].count; ++j) o = put_int(o, -(ev[i].index + j + 1));  // :1274
        }
    }
    o = put_int(o, 0);          // :1316
    memcpy(o, file_md5, 16);    // sendFiles :1148
    return RSH_OK;
}

int64_t rsh_generator_bytes(const rsh_header* h, const int32_t* weak, const uint8_t* strong, uint8_t* out, int64_t cap) {
    if (!h) return RSH_E_INVAL;
    const int64_t size = 16 + (int64_t)h->chunk_count * (4 + h->digest_length);
    if (!out) return size;
    if (cap < size || (h->chunk_count > 0 && (!weak || (!strong && h->digest_length > 0)))) return RSH_E_NOSPACE;
    uint8_t* o = out;
    o = put_int(o, h->chunk_count);  // Connection.sendChecksumHeader (Connection.java:40-45)
    o = put_int(o, h->block_length);
    o = put_int(o, h->digest_length);
    o = put_int(o, h->remainder);
    for (int32_t i = 0; i < h->chunk_count; ++i) {  // Generator.java:890-893
        o = put_int(o, weak[i]);
        memcpy(o, strong + (int64_t)i * h->digest_length, (size_t)h->digest_length);
        o += h->digest_length;
    }
    return size;
}

int rsh_dev_alloc(rsh_ctx* ctx, int64_t bytes, void** out) {
    if (!ctx || !out || bytes < 0) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    return hipMalloc(out, (size_t)(bytes ? bytes : 1)) == hipSuccess ? RSH_OK : RSH_E_NOMEM;
}

int rsh_dev_free(rsh_ctx* ctx, void* p) {
    if (!ctx) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    if (p) RSH_HIP(hipFree(p));
    return RSH_OK;
}

int rsh_memcpy_h2d(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (!ctx || bytes < 0 || (bytes > 0 && (!dst || !src))) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_memcpy_d2h(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (!ctx || bytes < 0 || (bytes > 0 && (!dst || !src))) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_debug_set_option(const char* name, int64_t value) {
    const int i = rsh::opt_index(name);
    if (!rsh::opt_settable(i)) return RSH_E_INVAL;  // unknown, or an A/B switch outside the diagnostics build
    rsh::opt_table()[i].store(value, std::memory_order_relaxed);
    return RSH_OK;
}

int rsh_debug_get_option(const char* name, int64_t* value) {
    const int i = rsh::opt_index(name);
    if (i < 0 || !value) return RSH_E_INVAL;
    *value = rsh::opt((rsh::Opt)i);
    return RSH_OK;
}

void rsh_debug_reset_options(void) {
    for (int i = 0; i < rsh::OPT_COUNT; ++i) rsh::opt_table()[i].store(rsh::opt_info()[i].def, std::memory_order_relaxed);
}

int rsh_debug_kernel_ms(rsh_ctx* ctx, int32_t which, double* ms) {
    if (!ctx || !ms || which < 0 || which > 1) return RSH_E_INVAL;
    *ms = -1.0;
    const bool timed = which == 0 ? ctx->gen_timed : ctx->spec_timed;
    if (!timed) return RSH_OK;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipEventSynchronize(which == 0 ? ctx->ev_gen_b : ctx->ev_k1b));
    float f = 0.f;
    RSH_HIP(hipEventElapsedTime(&f, which == 0 ? ctx->ev_gen_a : ctx->ev_k1a, which == 0 ? ctx->ev_gen_b : ctx->ev_k1b));
    *ms = f;
    return RSH_OK;
}

int rsh_debug_streams_busy(rsh_ctx* ctx, int32_t* mask) {
    if (!ctx || !mask) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    *mask = 0;
    const hipStream_t st[3] = {ctx->stream, ctx->aux, ctx->phase};
    for (int i = 0; i < 3; ++i) {
        const hipError_t e = hipStreamQuery(st[i]);
        if (e == hipErrorNotReady) *mask |= 1 << i;
        else if (e != hipSuccess) RSH_HIP(e);
    }
    return RSH_OK;
}

int rsh_debug_k1_clock(rsh_ctx* ctx, const void* d_data, int64_t n, int32_t block_length, int32_t reps,
                       double* clock_ghz) {
    if (!ctx || !d_data || !clock_ghz || reps <= 0 || block_length <= 0 || n <= 0 || block_length % 128 != 0 ||
        n % (64 * (int64_t)block_length) != 0)
        return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    const int64_t C = n / block_length;
    void *w = nullptr, *st = nullptr, *clk = nullptr;
    hipError_t e = hipMalloc(&w, (size_t)C * 4);
    if (e == hipSuccess) e = hipMalloc(&st, (size_t)C * 16);
    if (e == hipSuccess) e = hipMalloc(&clk, 16);
    if (e == hipSuccess) e = hipMemsetAsync(clk, 0, 16, ctx->stream);
    for (int32_t r = 0; e == hipSuccess && r < reps; ++r)
        e = rsh::launch_k1_clock(static_cast<const uint8_t*>(d_data), n, (uint32_t)block_length, 16, 0x04030201u,
                                 static_cast<int32_t*>(w), static_cast<uint8_t*>(st),
                                 static_cast<unsigned long long*>(clk), ctx->stream);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(h, clk, 16, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    for (void* p : {w, st, clk})
        if (p) (void)hipFree(p);
    RSH_HIP(e);
    *clock_ghz = h[1] ? 0.1 * (double)h[0] / (double)h[1] : 0.0;  // ticks / (ticks of 10 ns) / 10 ns -> GHz
    return RSH_OK;
}

int rsh_fill_splitmix_device(rsh_ctx* ctx, void* d_out, int64_t n, uint64_t key, int64_t byte_offset) {
    if (!ctx || (n > 0 && !d_out) || n < 0 || byte_offset < 0) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(rsh::launch_fill_splitmix(static_cast<uint8_t*>(d_out), n, key, byte_offset, ctx->stream));
    return RSH_OK;
}

}  // extern "C"
