// scan_backend.h -- the HIP implementation of the resolver's device services (resolver.h ScanBackend) for the
// single-file scans: scan_device (the file resident in HBM) and scan_tiled (HBM holding one tile at a time), both in
// scan.cpp, the only file that includes this one.  Each member answers one of the resolver's device questions with a
// round trip on the context's streams: range probes (first_hit, the batched flush chain), weak sums and bytes at
// positions, a window's digest, and the phase-shifted speculations (Sender.java:1282-1287).
#pragma once
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "ctx.h"
#include "device.h"
#include "host_md5.h"
#include "options.h"
#include "resolver.h"

namespace rshi {
// ------------------------------------------------------------------------------------------------
// HIP implementation of the resolver's services.
// ------------------------------------------------------------------------------------------------
constexpr size_t kFirstSlots = 1024;
hipError_t wait_stamp(const int* stamp, int gen, hipStream_t s);  // scan.cpp
// Device results to pinned host memory by a copy kernel (copy_few_kernel) rather than hipMemcpyAsync: between two
// kernels a D2H copy cost 47-100 us of idle queue (tools/queue_lat.hip case 8) where a kernel writing pinned memory
// cost none (case 9), and the profiler's async-copy tracing reported the copy engine's completions as never
// delivered.  The ranges travel in the kernel's arguments.  The kernel
// copies pinned host memory to the device as well (the segmented K1's descriptors, scan.cpp).
inline hipError_t copy_to_host(std::initializer_list<rsh::CopyEnt> ents, hipStream_t s) {
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
        rsh::ProbeOut* hf = pin<rsh::ProbeOut>(c_->h_first, 2);  // the record, then the copy's stamp
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
        F->nwin = guess ? 0 : kScanWindows;
        F->next_sums = guess ? 3 : 0;
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
        ok(rsh::launch_hit_window(F, hiv, req, 1, guess ? 0 : t_.chunk_count, rs_));
        // the results by one stamped workgroup; the host spins on the stamp (a stream synchronisation's wake-up
        // cost each probe round trip ~10-20 us more)
        rsh::CopyFew cf{};
        cf.e[cf.n++] = rsh::CopyEnt{reinterpret_cast<const uint8_t*>(d_first), reinterpret_cast<uint8_t*>(hf),
                                    (int64_t)sizeof(rsh::ProbeOut)};
        cf.e[cf.n++] = rsh::CopyEnt{c_->bucket.as<uint8_t>(), reinterpret_cast<uint8_t*>(hb),
                                    (int64_t)(rsh::HIT_BUCKET_INTS * sizeof(int32_t))};
        int* stamp = reinterpret_cast<int*>(hf + 1);
        const int sgen = c_->next_stamp();
        ok(rsh::launch_copy_few_stamped(cf, stamp, sgen, rs_));
        if (err == hipSuccess) ok(wait_stamp(stamp, sgen, rs_));
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
        if (guess) {  // no windows and no bucket came back: only T(p) and the next three windows' sums
            for (int64_t& w : win_pos_) w = -1;
            t_pos_ = (int64_t)hf->first;
            t_val_ = *reinterpret_cast<const int32_t*>(hh);
            guess_pos_ = t_pos_;
            memcpy(guess_sums_, hh + 4, sizeof(guess_sums_));
            t_.prime_clear();
            return t_pos_;
        }
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
    // The phase guess's probes (scan.cpp): no hit windows and no bucket, but T(p + k B), k = 1..3, of the hit in the
    // same round trip (hit_window_kernel, ScanFile::next_sums) -- the guess checks four consecutive windows
    bool guess = false;
    int64_t guess_pos_ = -1;
    int32_t guess_sums_[3] = {0, 0, 0};
    bool guess_sums(int64_t p, int32_t out[3]) const {
        if (p != guess_pos_) return false;
        memcpy(out, guess_sums_, sizeof(guess_sums_));
        return true;
    }
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
        ph_gen_ = c_->next_gen();
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
            note_error(e, line, "scan_backend.h");
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

}  // namespace rshi
