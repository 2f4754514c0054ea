// resolver.cpp -- sequential Sender state machine over device-computed events (see resolver.h).
// Reference: session/Sender.java:1235-1327 (loop), session/Checksum.java:175-276 (candidate order),
// io/FileView.java:143-185,235-278 (window, mark, isFull), util/Rolling.java:25-60 (add/subtract).
#include "resolver.h"

#include "options.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <limits>

namespace rsh {

HostTimes& host_times() {
    static thread_local HostTimes t;
    return t;
}

namespace {
// Option scan_trace = 1: one stderr line per host-side table operation (=2: totals only, see host_times)
struct HostTrace {
    const char* what;
    int64_t arg;
    double* acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    HostTrace(const char* w, int64_t a, double* total) : what(w), arg(a), acc(total) {}
    ~HostTrace() {
        const int on = (int)opt(OPT_SCAN_TRACE);
        if (!on) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        *acc += ms;
        if (on == 1) fprintf(stderr, "[rsh] %-10s %10lld %9.3f ms\n", what, (long long)arg, ms);
    }
};
}  // namespace

void ChunkTable::build() {
    HostTrace tr("tab_index", chunk_count, &host_times().sort_ms);
    if (indexed_) return;
    const auto t0 = std::chrono::steady_clock::now();
    const int32_t n = chunk_count;
    weak_copy_.assign(weak, weak + n);
    weak = weak_copy_.data();
    uint32_t slots = 1u << 10;
    while (slots < 2u * (uint32_t)n && slots < (1u << 30)) slots <<= 1;
    index_mask_ = slots - 1;
    head_.assign(slots, -1);
    next_.resize((size_t)n);
    for (int32_t i = n - 1; i >= 0; --i) {  // prepend in descending order: chains ascend
        const uint32_t h = ((uint32_t)weak[i] * 0x9E3779B1u >> 7) & index_mask_;
        next_[(size_t)i] = head_[h];
        head_[h] = i;
    }
    indexed_ = true;
    sort_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

const int32_t* ChunkTable::bucket(int32_t key, int32_t* size) {
    for (int k = 0; k < primed_n_; ++k)
        if (primed_[(size_t)k].key == key) {
            *size = (int32_t)primed_[(size_t)k].idx.size();
            return primed_[(size_t)k].idx.data();
        }
    HostTrace tr("bucket", key, &host_times().bucket_ms);
    if (!indexed_ && scan_lookups_ >= kScanLookups) build();
    scratch_.clear();
    if (indexed_) {
        for (int32_t i = head_[((uint32_t)key * 0x9E3779B1u >> 7) & index_mask_]; i >= 0; i = next_[(size_t)i])
            if (weak[i] == key) scratch_.push_back(i);
        *size = (int32_t)scratch_.size();
        return scratch_.data();
    }
    ++scan_lookups_;
    int32_t cnt = 0;  // counting pass (vectorises); most lookups find nothing
    for (int32_t i = 0; i < chunk_count; ++i) cnt += weak[i] == key;
    if (cnt) {
        scratch_.reserve(cnt);
        for (int32_t i = 0; i < chunk_count; ++i)
            if (weak[i] == key) scratch_.push_back(i);
    }
    *size = cnt;
    return scratch_.data();
}

void ChunkTable::keys_with_digest(const uint8_t* d, std::vector<int32_t>* keys) const {
    HostTrace tr("dkeys", chunk_count, &host_times().dkeys_ms);
    keys->clear();
    const int64_t dl = digest_length;
    if (dl == 0) {  // every chunk carries the empty digest
        keys->assign(weak, weak + chunk_count);
    } else {
        const uint8_t d0 = d[0];
        const uint8_t* sp = strong;
        for (int32_t i = 0; i < chunk_count; ++i, sp += dl)  // first-byte filter, then the full compare
            if (sp[0] == d0 && memcmp(sp, d, (size_t)dl) == 0) keys->push_back(weak[i]);
    }
    std::sort(keys->begin(), keys->end());
    keys->erase(std::unique(keys->begin(), keys->end()), keys->end());
}

namespace {

inline uint32_t lo16(int32_t v) { return (uint32_t)v & 0xFFFFu; }
inline uint32_t hi16(int32_t v) { return (uint32_t)v >> 16; }
inline int32_t pack16(uint32_t lo, uint32_t hi) { return (int32_t)((lo & 0xFFFFu) | (hi << 16)); }
inline int32_t jbyte(uint8_t v) { return (int32_t)(int8_t)v; }
inline int32_t roll_sub(int32_t cs, int32_t w, uint8_t x) {  // Rolling.java:56-60
    return pack16(lo16(cs) - (uint32_t)jbyte(x), hi16(cs) - (uint32_t)w * (uint32_t)jbyte(x));
}
inline int32_t roll_add(int32_t cs, uint8_t x) {  // Rolling.java:25-29
    const uint32_t lo = lo16(cs) + (uint32_t)jbyte(x);
    return pack16(lo, hi16(cs) + lo);
}

// Checksum.java:175-195 binarySearch + :206-213 closeIndexOf over one bucket (ascending chunk index).
int32_t close_index_of(const int32_t* bucket, int32_t size, int32_t chunk_index) {
    int32_t l = 0, r = size - 1;
    while (l <= r) {
        const int32_t m = l + (r - l) / 2;
        if (bucket[m] == chunk_index) return m;
        if (bucket[m] < chunk_index) l = m + 1;
        else r = m - 1;
    }
    return l < size - 1 ? l : size - 1;
}

}  // namespace

namespace {
// Index of the first of `count` elements of `esize` bytes at which a and b differ (count if none): memcmp over
// 4 KiB blocks, then the block that differs element by element.
int64_t first_mismatch(const void* a, const void* b, int64_t count, int64_t esize) {
    const uint8_t* x = static_cast<const uint8_t*>(a);
    const uint8_t* y = static_cast<const uint8_t*>(b);
    const int64_t per = std::max<int64_t>(1, 4096 / esize);
    for (int64_t i = 0; i < count; i += per) {
        const int64_t m = std::min(per, count - i);
        if (memcmp(x + i * esize, y + i * esize, (size_t)(m * esize)) == 0) continue;
        for (int64_t j = i;; ++j)
            if (memcmp(x + j * esize, y + j * esize, (size_t)esize) != 0) return j;
    }
    return count;
}
}  // namespace

void flush_positions(const FlushChain& q, std::vector<int64_t>* tpos, std::vector<int64_t>* bpos) {
    tpos->clear();
    bpos->clear();
    for (int64_t i = 0; i < q.K; ++i) {
        const int64_t fi = q.f + 10 * q.B * i;
        tpos->push_back(fi);
        tpos->push_back(fi + q.B);
        bpos->push_back(fi);
        bpos->push_back(fi + 2 * q.B - 1 < q.n ? fi + 2 * q.B - 1 : fi);
    }
}

void flush_intervals(const FlushChain& q, std::vector<FlushStep>* steps, std::vector<ProbeInterval>* ivs) {
    steps->clear();
    ivs->clear();
    for (int64_t i = 0; i < q.K; ++i) {
        const int64_t s2 = q.f + 10 * q.B * i + q.B;
        steps->push_back(FlushStep{s2, 0u, 0u});
        if (s2 > q.last) break;
        const int64_t fn = (s2 + 10 * q.B <= q.n) ? s2 + 9 * q.B : std::numeric_limits<int64_t>::max();
        ivs->push_back(ProbeInterval{s2, std::min(fn, q.last) + 1, s2, 0u, 0u});
    }
}

// The flush bookkeeping of Sender.java:1294-1310 from the rolling value R at each flush point (quirk A): the Java
// code subtracts x_f with the full window, slides by B, adds the window's new last byte only when the window is
// still full, and keeps rolling the old value -- so after flush i the desync is E_i = R2_i - T(s2_i).
void flush_chain_host(const FlushChain& q, const int32_t* tv, const uint8_t* bv, std::vector<FlushStep>* steps,
                      std::vector<ProbeInterval>* ivs) {
    flush_intervals(q, steps, ivs);
    const int64_t B = q.B, n = q.n, last = q.last;
    auto clampB = [&](int64_t p) { return std::min<int64_t>(p, n - B); };
    int32_t R = pack16(lo16(tv[0]) + q.el, hi16(tv[0]) + q.eh);
    for (size_t i = 0; i < steps->size(); ++i) {
        FlushStep& stp = (*steps)[i];
        const int32_t R1 = roll_sub(R, (int32_t)B, bv[2 * i]);
        int32_t R2 = R1;
        if (stp.s2 <= last && std::min<int64_t>(B, n - stp.s2) == B) R2 = roll_add(R1, bv[2 * i + 1]);  // :1308-1310
        const int32_t T2 = tv[2 * i + 1];
        stp.elo = (lo16(R2) - lo16(T2)) & 0xFFFFu;
        stp.ehi = (hi16(R2) - hi16(T2)) & 0xFFFFu;
        if (i < ivs->size()) {
            (*ivs)[i].e_lo = stp.elo;
            (*ivs)[i].e_hi = stp.ehi;
        }
        if (stp.s2 > last) break;
        if ((int64_t)i + 1 < q.K) {  // the rolling value at the next flush point
            const int64_t fn = (stp.s2 + 10 * B <= n) ? stp.s2 + 9 * B : std::numeric_limits<int64_t>::max();
            const uint32_t ehi2 = stp.ehi + stp.elo * (uint32_t)(clampB(fn) - clampB(stp.s2));
            R = pack16(lo16(tv[2 * i + 2]) + stp.elo, hi16(tv[2 * i + 2]) + ehi2);
        }
    }
}

int64_t ScanBackend::flush_probe(const ProbeInterval* pre, int64_t npre, const FlushChain& q,
                                 std::vector<FlushStep>* steps, std::vector<ProbeInterval>* ivs,
                                 const std::vector<int32_t>* keys) {
    std::vector<int64_t> tpos, bpos;
    flush_positions(q, &tpos, &bpos);
    std::vector<int32_t> tv(tpos.size());
    std::vector<uint8_t> bv(bpos.size());
    flush_gather(tpos.data(), (int64_t)tpos.size(), tv.data(), bpos.data(), (int64_t)bpos.size(), bv.data());
    flush_chain_host(q, tv.data(), bv.data(), steps, ivs);
    std::vector<ProbeInterval> all(pre, pre + npre);
    all.insert(all.end(), ivs->begin(), ivs->end());
    return all.empty() ? -1 : first_hit(all.data(), (int64_t)all.size(), keys);
}

bool resolve_run(int64_t n, ChunkTable& table, ScanBackend& be, ResolveState* state, ResolveResult* out,
                 const std::function<bool()>& yield) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t B = table.block_length;
    const int dl = table.digest_length;
    const int64_t S = table.remainder > 0 ? table.remainder : B;  // getSmallestChunkSize, Checksum.java:131-137
    const int64_t last = n - S;  // visited positions satisfy wl(s) >= S  <=>  s <= n - S
    const int64_t nB = n - B;
    // the speculation the backend has now (none while it is still in flight: every lookup below then
    // takes the generic path, which gives the same answer); re-read every step, since a tiled backend
    // extends it as its tiles land
    // The aligned sums are asked for only when a step needs them (NAL()): an aligned run of matches resolves from
    // the chain flags alone, and a backend may bring the sums to the host only on request (HipBackend).
    int64_t nal_step = -1, nflags = 0, max_batch = 1;
    const int32_t* aw = nullptr;
    const uint8_t* as = nullptr;
    const uint8_t* fl = nullptr;
    auto NAL = [&]() -> int64_t {
        if (nal_step < 0) {
            nal_step = be.aligned_count();
            aw = be.aligned_weak();
            as = be.aligned_strong();
        }
        return nal_step;
    };
    auto refresh = [&] {
        nal_step = -1;
        fl = be.chain_flags();
        nflags = std::min<int64_t>(be.flags_count(), table.chunk_count);
        max_batch = be.max_batch();
    };
    refresh();
    auto wl = [&](int64_t s) { return std::min<int64_t>(B, n - s); };  // FileView window length
    auto clampB = [&](int64_t p) { return std::min<int64_t>(p, nB); };

    std::vector<rsh_event>& ev = out->ev;
    rsh_scan_stats& st = out->stats;
    auto emit_lit = [&](int64_t off, int64_t len) {  // sendDataFrom; zero-length calls write nothing
        if (len <= 0) return;
        ev.push_back(rsh_event{off, len, RSH_EV_LITERAL, 0, 0, 0});
        out->literal += len;
    };
    auto emit_match = [&](int64_t off, int64_t len, int32_t idx, int32_t cnt) {
        if (!ev.empty()) {
            rsh_event& b = ev.back();
            if (b.kind == RSH_EV_MATCH && b.index + b.count == idx && b.offset + b.length == off) {
                b.count += cnt;
                b.length += len;
                out->matched += len;
                return;
            }
        }
        ev.push_back(rsh_event{off, len, RSH_EV_MATCH, idx, cnt, 0});
        out->matched += len;
    };

    // Sender state (file coordinates), kept in *state between calls
    int64_t& s = state->s;
    int64_t& m = state->m;
    int32_t& pref = state->pref;
    uint32_t& elo = state->elo;
    uint32_t& ehi = state->ehi;
    int64_t& anchor = state->anchor;
    bool& md5c_valid = state->md5c_valid;
    state->md5c.resize((size_t)dl);
    uint8_t* md5c = state->md5c.data();
    std::vector<int32_t>& dkeys = state->dkeys;
    bool& dkeys_ready = state->dkeys_ready;
    int64_t& batch = state->batch;
    if (state->done) return true;

    auto E_at = [&](int64_t p, uint32_t* lo, uint32_t* hi) {
        *lo = elo;
        *hi = ehi + elo * (uint32_t)(clampB(p) - clampB(anchor));
    };
    auto T_at = [&](int64_t p) -> int32_t {
        if (p % B == 0 && p / B < NAL()) return aw[p / B];
        return be.weak_at(p);
    };
    // FileView flush at f (isFull, Sender.java:1294-1302) with rolling value R at f: the Java code
    // subtracts x_f with the full window, slides by B and keeps rolling the old value.
    auto flush = [&](int64_t f, int32_t R) {
        emit_lit(m, f + B - m);
        st.flushes++;
        const int32_t R1 = roll_sub(R, (int32_t)B, be.byte_at(f));
        const int64_t s2 = f + B;
        m = s2;
        s = s2;
        if (s2 <= last) {
            int32_t R2 = R1;
            if (wl(s2) == B) R2 = roll_add(R1, be.byte_at(s2 + B - 1));  // :1308-1310
            const int32_t T2 = T_at(s2);
            elo = (lo16(R2) - lo16(T2)) & 0xFFFFu;
            ehi = (hi16(R2) - hi16(T2)) & 0xFFFFu;
            anchor = s2;
        }
    };

    auto elapsed = [&] {
        st.resolver_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    // The batched flush chain from the flush point f.  No candidate before f: speculate that none occurs in the
    // next K flush intervals either -- their flush points are f + 10B i (FileView.isFull at mark + 9B), the rolling
    // value's desync E after each one is a closed-form function of T and two bytes at the flush (flush_chain_host)
    // -- so one gather, the chain and one probe over all K intervals replace K round trips (the GPU backends do all
    // three in one).  K doubles while no event turns up (wasted probing <= 2x).  The doubling starts higher when
    // candidates are rare: a stale digest carried by few chunks leaves about |keys| 10B / 2^32 candidate positions
    // per interval (x4 for the weak sums' uneven spread), so a poisoned state with a handful of keys probes
    // thousands of intervals at once instead of climbing from one through a dozen round trips.  The batch size only
    // decides how much is speculated per probe, never the result.
    auto flush_chain_at = [&](int64_t f, const std::vector<int32_t>* keys) -> FlushChain {
        const int64_t nkeys = keys ? (int64_t)keys->size() : (int64_t)table.chunk_count;
        const int64_t floor_k = std::clamp<int64_t>((int64_t)((1ull << 32) / ((uint64_t)(40 * B) * (uint64_t)std::max<int64_t>(nkeys, 1))), 1, 4096);
        batch = std::max(batch, floor_k);
        int64_t K = 1;
        const int64_t kcap = std::min(max_batch, be.max_batch_at(f));
        while (K < std::min(batch, kcap) && f + 10 * B * K + B <= n) ++K;
        FlushChain q;
        q.f = f, q.K = K, q.B = B, q.n = n, q.last = last;
        E_at(f, &q.el, &q.eh);
        return q;
    };
    // One round: the intervals pre (E known, ending at pre_end) and the chain's.  A hit inside pre is left in
    // pre_hit for the caller (returns false); otherwise every flush before the interval holding the hit (all of
    // them without one) is committed and true is returned.
    int64_t pre_hit = -1;
    auto flush_round = [&](const ProbeInterval* pre, int64_t npre, const FlushChain& q, const std::vector<int32_t>* keys,
                           int64_t pre_end) -> bool {
        std::vector<FlushStep> chain;
        std::vector<ProbeInterval> iv;
        const int64_t hit = be.flush_probe(pre, npre, q, &chain, &iv, keys);
        if (npre > 0 || !iv.empty()) st.probe_launches++;
        if (npre > 0 && hit >= 0 && hit <= pre_end) {
            pre_hit = hit;
            return false;
        }
        // commit every flush whose following interval holds no candidate
        int64_t commit = (int64_t)chain.size();
        if (hit >= 0)
            for (size_t j = 0; j < iv.size(); ++j)
                if (hit >= iv[j].a && hit < iv[j].b) {
                    commit = (int64_t)j + 1;  // flushes 0..j happen before the event
                    break;
                }
        for (int64_t i = 0; i < commit; ++i) {
            emit_lit(m, 10 * B);
            st.flushes++;
            m = s = chain[(size_t)i].s2;
            elo = chain[(size_t)i].elo;
            ehi = chain[(size_t)i].ehi;
            anchor = s;
        }
        batch = hit >= 0 ? 1 : std::min<int64_t>(batch * 2, 4096);
        return true;
    };
    while (s <= last) {
        if (yield && yield()) {  // between two steps: the caller resumes with the same state
            elapsed();
            return false;
        }
        refresh();
        const bool synced = (elo == 0 && ehi == 0);
        // (1) aligned chain: preferred index == k and source window k carries chunk k's sums.
        if (!md5c_valid && synced && s % B == 0) {
            const int64_t k = s / B;
            if (k == pref && k < nflags && fl[k]) {
                // the run ends at the first unset flag (memchr), or where the windows reach past `last`: each
                // window at p <= last is min(B, n - p) long, so t windows from s end at min(n, s + t B) and
                // the walk stops once that exceeds last (a per-window loop took ~0.1 ms for 131072 windows)
                const void* z = memchr(fl + k, 0, (size_t)(nflags - k));
                const int64_t j_end = z ? (int64_t)(static_cast<const uint8_t*>(z) - fl) : nflags;
                const int64_t t_max = (last - s) / B + 1;  // windows starting at s, s + B, ... <= last
                const int64_t t = std::min<int64_t>(j_end - k, t_max);
                const int64_t j = k + t, p = std::min<int64_t>(n, s + t * B);
                emit_lit(m, s - m);
                emit_match(s, p - s, (int32_t)k, (int32_t)(j - k));
                st.chain_matches += j - k;
                s = p;
                m = p;
                pref = (int32_t)j;
                anchor = s;
                continue;
            }
        }
        // (1') chain at any other phase, or aligned with pref != k: the window at s is matched against chunk
        // pref exactly when its sums are pref's (T(s) == weak[pref] puts pref in the bucket, so closeIndexOf
        // makes it the first candidate, Checksum.java:206-213, and its digest then decides, Sender.java:1265),
        // and the match jumps a whole window (:1282), so the next window is s + w against pref + 1.
        if (!md5c_valid && synced && pref < table.chunk_count) {
            PhaseView pv;
            bool have = false;
            if (s % B == 0 && s / B < NAL()) {
                pv.s0 = 0, pv.count = NAL(), pv.w = aw, pv.st = as;
                have = true;
            } else if (s % B != 0) {
                const bool chain = !ev.empty() && ev.back().kind == RSH_EV_MATCH && ev.back().count >= 2 &&
                                   ev.back().offset + ev.back().length == s;
                have = be.phase_sums(s, chain, &pv);
            }
            if (have) {
                // windows s + iB (i < t) against chunks pref + i while both sums agree: the first weak and the
                // first digest mismatch over the contiguous arrays (block memcmp; a per-window loop took ~0.5 ms
                // for a 131072-window phase chain), capped at the windows that start at or before `last`
                const int64_t k0 = (s - pv.s0) / B, C = table.chunk_count;
                const int64_t lim = std::max<int64_t>(0, std::min({pv.count - k0, C - (int64_t)pref, (last - s) / B + 1}));
                int64_t t = first_mismatch(pv.w + k0, table.weak + pref, lim, 4);
                if (dl > 0 && t > 0) t = std::min(t, first_mismatch(pv.st + k0 * dl, table.strong + (int64_t)pref * dl, t, dl));
                const int64_t c = pref + t, p = std::min<int64_t>(n, s + t * B);
                if (c > pref) {
                    emit_lit(m, s - m);
                    emit_match(s, p - s, pref, (int32_t)(c - pref));
                    st.phase_matches += c - pref;
                    s = p;
                    m = p;
                    pref = (int32_t)c;
                    anchor = s;
                    continue;
                }
            }
        }
        // (2) next candidate event in [s, stop]: the first flush point bounds the state's validity.
        const int64_t f = (m + 10 * B <= n) ? m + 9 * B : std::numeric_limits<int64_t>::max();
        const int64_t stop = std::min(f, last);
        const std::vector<int32_t>* keys = nullptr;
        bool none = false;
        if (md5c_valid) {  // stale digest: only chunks whose digest is md5c can ever match
            if (!dkeys_ready) {
                table.keys_with_digest(md5c, &dkeys);
                dkeys_ready = true;
            }
            keys = &dkeys;
            none = dkeys.empty();
        }
        if (none) {
            // Stale digest that no chunk carries: no candidate can ever match again, so md5c and the
            // state never change; only the flushes at mark + 9B remain (closed form, no device work).
            while (m + 10 * B <= n) {
                emit_lit(m, 10 * B);
                m += 10 * B;
                st.flushes++;
            }
            s = m;
            break;
        }
        int64_t p = -1;
        if (!none) {
            int64_t a = s;
            if (!md5c_valid && synced && s % B == 0 && s / B < NAL()) {  // key known from aligned sums
                int32_t size;
                table.bucket(aw[s / B], &size);
                if (size > 0) p = s;
                else a = s + 1;
            }
            const bool clear = state->clear_from == s && state->clear_to >= stop;  // the walk searched it
            if (p < 0 && a <= stop && !clear) {
                uint32_t el, eh;
                E_at(a, &el, &eh);
                const ProbeInterval one{a, stop + 1, a, el, eh};
                if (md5c_valid && f <= last && be.one_round(a, f)) {
                    // A stale digest's few keys: an event before the flush point is unlikely, so the batched flush
                    // chain after it (below) is probed in the same round trip, this interval first (when the backend
                    // can answer both from one tile; else [a, stop] alone first, then the chain below).
                    const FlushChain q = flush_chain_at(f, keys);
                    state->clear_from = state->clear_to = -1;
                    if (flush_round(&one, 1, q, keys, stop)) continue;  // no event in [a, stop]: flushes committed
                    p = pre_hit;
                } else {
                    p = be.first_hit(&one, 1, keys);
                    st.probe_launches++;
                }
            }
        }
        state->clear_from = state->clear_to = -1;
        if (p >= 0) {
            uint32_t el, eh;
            E_at(p, &el, &eh);
            const int32_t T = T_at(p);
            const int32_t R = pack16(lo16(T) + el, hi16(T) + eh);
            const int64_t w = wl(p);
            st.events++;
            int32_t size;
            const int32_t* bk = table.bucket(R, &size);
            int32_t hit = -1;
            if (size > 0) {  // getCandidateChunks order (Checksum.java:215-276)
                const int32_t init = close_index_of(bk, size, pref);
                for (int32_t it = -1; it < size; ++it) {
                    int32_t pos;
                    if (it < 0) {
                        pos = init;
                    } else {
                        if (it == init || table.chunk_length(bk[it]) != w) continue;
                        pos = it;
                    }
                    const int32_t c = bk[pos];
                    if (!md5c_valid) {  // Sender.java:1259-1263
                        PhaseView pd;
                        if (p % B == 0 && p / B < NAL()) {
                            memcpy(md5c, as + (p / B) * dl, (size_t)dl);
                        } else if (p % B != 0 && be.phase_sums(p, false, &pd)) {  // a landed phase speculation's
                            memcpy(md5c, pd.st + ((p - pd.s0) / B) * dl, (size_t)dl);  // digest of this window
                        } else {
                            uint8_t full[16];
                            be.md5_at(p, full);
                            memcpy(md5c, full, (size_t)std::min(dl, 16));
                            if (dl > 16) memset(md5c + 16, 0, (size_t)(dl - 16));
                            st.host_md5_windows++;
                        }
                        md5c_valid = true;
                        dkeys_ready = false;
                    }
                    if (memcmp(md5c, table.strong + (int64_t)c * dl, (size_t)dl) == 0) {
                        hit = c;
                        break;
                    }
                }
            }
            batch = 1;
            if (hit >= 0) {  // Sender.java:1265-1288
                emit_lit(m, p - m);
                emit_match(p, w, hit, 1);
                pref = hit + 1;
                s = p + w;
                m = s;
                elo = ehi = 0;
                anchor = s;
                md5c_valid = false;
                dkeys_ready = false;
                if (s % B != 0 && s <= last) be.phase_hint(s);
                continue;
            }
            if (p == f) flush(p, R);
            else s = p + 1;
            continue;
        }
        if (f <= last) {
            // No candidate before the flush point: the batched flush chain (flush_round above)
            flush_round(nullptr, 0, flush_chain_at(f, keys), keys, -1);
            continue;  // the loop re-finds the event (if any) in [s, stop] and resolves it
        }
        break;
    }
    emit_lit(m, n - m);  // Sender.java:1313-1316 (firstOffset == mark once the loop ends)
    state->done = true;
    elapsed();
    return true;
}

void resolve_scan(int64_t n, ChunkTable& table, ScanBackend& be, ResolveResult* out) {
    ResolveState state;
    resolve_run(n, table, be, &state, out, nullptr);
}

}  // namespace rsh
