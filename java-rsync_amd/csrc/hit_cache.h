// hit_cache.h -- a range probe's hit list (ProbeOut, written by probe_first_kernel) and the host cache
// that answers the resolver's follow-up probes from it.  No HIP types: the CPU test backend uses it too.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "resolver.h"

namespace rsh {

constexpr int PROBE_HITS_CAP = 64;
// A probe's answer: the first hitting position (~0 if none) and, while there are at most PROBE_HITS_CAP
// of them, every hitting position with its key (unordered).  The caller presets first = ~0, count = 0.
struct ProbeOut {
    unsigned long long first;
    unsigned long long count;
    unsigned long long pos[PROBE_HITS_CAP];
    uint32_t key[PROBE_HITS_CAP];
};

// Windows the hit kernel returns with a probe: slot k holds the window at the k-th smallest listed hit
// (slot 0: the first hit, always; slots >= 1 only when the list is complete), for k < the file's nwin
// (ScanFile::nwin <= HIT_WINDOWS).  More slots trade D2H bytes and host digests for round trips: the
// single-file scan asks for 2 (the second digest is computed on a host thread while the resolver handles
// the first hit); the batched scan asks for 1 -- on config 4 (128 x 128 MiB) 4 slots cut the rounds from
// 26 to 18 but gave no faster step on 50%-modified bases and a slower one on identical bases (host
// digests of windows the speculation would have supplied).
constexpr int HIT_WINDOWS = 4;
// ScanFile::next_sums at most: the hit buffer's 16-B header holds T(p) and T(p + k B), k = 1..3.
constexpr int NEXT_SUMS_MAX = 3;
// Buckets of the listed hits' keys computed with the probe (HitBuckets region of ScanFile::bucket): up
// to LISTED_IDX chunk indices per listed key, in no particular order.
constexpr int LISTED_IDX = 3;
inline void window_slots(const ProbeOut& o, int nwin, int64_t (&slot)[HIT_WINDOWS]) {
    for (int k = 0; k < HIT_WINDOWS; ++k) slot[k] = -1;
    if (o.first == ~0ull) return;
    slot[0] = (int64_t)o.first;
    if (o.count > (unsigned long long)PROBE_HITS_CAP) return;
    std::vector<int64_t> p(o.pos, o.pos + o.count);
    std::sort(p.begin(), p.end());
    for (int k = 1; k < nwin && k < HIT_WINDOWS && k < (int)p.size(); ++k) slot[k] = p[(size_t)k];
}

// The hits of the last single-interval range probe.  A later probe of [a', b') with the same key function
// E and key set, starting inside the probed range, is answered from the list without a device round trip
// when the list covers it, or is cut to the part beyond the probed range (the answer is the same: the
// list proves [a', b) hit-free).  Typical use: after a match at p the resolver asks for the first hit
// in [p + B, m' + 9B]; the previous probe already covered most of that range.
struct HitCache {
    bool valid = false;
    int64_t a = 0, b = 0;        // probed range [a, b)
    bool complete = false;       // every hit in [a, b) is listed (else only the first one)
    uint32_t e_lo = 0, e_c = 0;  // key function: E(p) = (e_lo, e_c + e_lo * min(p, n - B)) mod 2^16
    bool full_table = true;      // key set: the whole received table, or `keys`
    std::vector<int32_t> keys;
    std::vector<std::pair<int64_t, uint32_t>> hits;  // (position, key), ascending
    int64_t nB = 0;              // n - B

    uint32_t e_const(const ProbeInterval& iv) const {
        return (iv.e_hi - iv.e_lo * (uint32_t)std::min(iv.anchor, nB)) & 0xFFFFu;
    }
    bool same_function(const ProbeInterval& iv, const std::vector<int32_t>* ks) const {
        if (!valid || (iv.e_lo & 0xFFFFu) != e_lo || e_const(iv) != e_c) return false;
        if (full_table != (ks == nullptr)) return false;
        return full_table || *ks == keys;
    }
    // T(p) from the key that hit at p
    int32_t weak_of(int64_t p, uint32_t key) const {
        const uint32_t eh = e_c + e_lo * (uint32_t)std::min(p, nB);
        return (int32_t)((((key & 0xFFFFu) - e_lo) & 0xFFFFu) | ((((key >> 16) - eh) & 0xFFFFu) << 16));
    }
    // 1: answered (*p = first hit in [iv.a, iv.b) or -1, *T = its weak sum); 0: probe [*a2, iv.b) instead.
    int lookup(const ProbeInterval& iv, const std::vector<int32_t>* ks, int64_t* p, int32_t* T,
               int64_t* a2) const {
        *a2 = iv.a;
        if (!same_function(iv, ks) || iv.a < a || iv.a > b) return 0;
        auto it = std::lower_bound(hits.begin(), hits.end(), std::make_pair(iv.a, (uint32_t)0));
        if (!complete) {  // only the range's first hit is known; it answers iff it lies at or after iv.a
            if (it == hits.begin() && it != hits.end() && it->first < iv.b) {
                *p = it->first;
                *T = weak_of(it->first, it->second);
                return 1;
            }
            return 0;
        }
        if (it != hits.end() && it->first < iv.b) {
            *p = it->first;
            *T = weak_of(it->first, it->second);
            return 1;
        }
        if (iv.b <= b) {
            *p = -1;
            return 1;
        }
        *a2 = b;
        return 0;
    }
    // After a probe over several intervals (the batched flush chain): the resolver's next question is the
    // first hit inside the interval that holds the first hit, with that interval's key function -- keep
    // that interval's hits (all of them when the list is complete, else the first).  Without a hit every
    // flush is committed and the next question is the last interval itself: keep it, proven hit-free.
    void fill_batch(const ProbeInterval* iv, int64_t count, const std::vector<int32_t>* ks, const ProbeOut& o,
                    int64_t n_minus_B) {
        valid = false;
        if (count <= 0) return;
        if (o.first == ~0ull) {
            fill(iv[count - 1], ks, o, n_minus_B);
            return;
        }
        const int64_t p = (int64_t)o.first;
        for (int64_t j = 0; j < count; ++j) {
            if (p < iv[j].a || p >= iv[j].b) continue;
            ProbeOut one = o;  // the listed hits of interval j only (keys follow each interval's own E)
            if (o.count <= (unsigned long long)PROBE_HITS_CAP) {
                one.count = 0;
                for (unsigned long long i = 0; i < o.count; ++i)
                    if ((int64_t)o.pos[i] >= iv[j].a && (int64_t)o.pos[i] < iv[j].b) {
                        one.pos[one.count] = o.pos[i];
                        one.key[one.count] = o.key[i];
                        ++one.count;
                    }
            }
            fill(iv[j], ks, one, n_minus_B);
            return;
        }
    }
    void fill(const ProbeInterval& iv, const std::vector<int32_t>* ks, const ProbeOut& o, int64_t n_minus_B) {
        nB = n_minus_B;
        valid = true;
        a = iv.a;
        b = iv.b;
        e_lo = iv.e_lo & 0xFFFFu;
        e_c = e_const(iv);
        full_table = ks == nullptr;
        if (ks) keys = *ks;
        else keys.clear();
        hits.clear();
        complete = o.count <= (unsigned long long)PROBE_HITS_CAP;
        if (complete) {
            for (unsigned long long i = 0; i < o.count; ++i) hits.emplace_back((int64_t)o.pos[i], o.key[i]);
            std::sort(hits.begin(), hits.end());
        } else if (o.first != ~0ull) {
            for (unsigned long long i = 0; i < (unsigned long long)PROBE_HITS_CAP; ++i)
                if (o.pos[i] == o.first) hits.emplace_back((int64_t)o.first, o.key[i]);
            if (hits.empty()) valid = false;  // the first hit's key was not listed
            else hits.resize(1);
        }
    }
};

}  // namespace rsh
