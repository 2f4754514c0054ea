// device_chain.hip -- gfx950 kernels of the batched scan's chain walk (batch.cpp): one workgroup per file advances
// its Sender (Sender.java:1235-1327) through runs of aligned matches, flushes and closed-form literal stretches on the
// device, searching tiles of positions against the file's key set in LDS and digesting hit windows; helper
// workgroups map later tiles ahead of slow walks (the hit map); the chunk index the walks look buckets up in.  The
// probes are in device_scan.hip, the K1 kernels in device.hip.  See DESIGN.md section 5a.
#include <hip/hip_runtime.h>

#include "device.h"
#include "device_common.h"
#include "device_roll.h"
#include "md5_core.h"
#include "options.h"

#include <algorithm>
#include <type_traits>

namespace rsh {

// ------------------------------------------------------------------------------------------------
// Chain advance (batched Sender scan, batch.cpp): one workgroup per file walks Sender.sendMatchesAndData
// (Sender.java:1235-1327) on the device for as long as the state stays synced (no FileView flush since the last
// match, so R = T) and unpoisoned (localChunkMd5sum == null, :1248) and every candidate digest comes from the
// aligned speculation -- the resolver's steps (1), (1') at aligned positions and (2) (resolver.cpp), with the
// candidate order of Checksum.getCandidateChunks (:206-276).  Anything else (a flush, a hit at an unaligned
// position, a digest mismatch that poisons the cached digest, a bucket longer than CHAIN_BUCKET_CAP, the
// shrinking windows at the end of a file with a remainder, a full event buffer) stops the walk before that step:
// the host resolver resumes from the returned state and takes the step itself.  So the device emits exactly
// the events the resolver would, in the same order.  In config 4's 50%-modified form (every other block
// replaced) a file's run of MATCH / LIT pairs until its first false weak hit cost one device round trip per
// pair on the host path; here the whole run is one launch for every file of the segment.
//
// All lanes keep the same copy of the state (s, mark, pref) and take the same decisions (every value they
// branch on is read from global memory or LDS by all of them); lane 0 writes the events.
// ------------------------------------------------------------------------------------------------
// CHAIN_THREADS, CHAIN_PPT, CHAIN_TILE, CHAIN_SEGS: device.h (the host sizes the hit map with them)
constexpr int CHAIN_EV_LDS = 64;  // events a walk holds in LDS before writing them out
// The walk's section timers (ChainOut::t_*, ChainHelp::t_*: the scan_trace report) read the wall clock only when the
// launch is traced: each read is a scalar memory operation the walk's next LDS wait also waits for.  Build with
// -DRSH_CHAIN_TIMERS_ALWAYS for the A/B of the timers' own cost.
__device__ __forceinline__ int64_t chain_clock(bool timed) {
#ifdef RSH_CHAIN_TIMERS_ALWAYS
    timed = true;
#endif
    return timed ? (int64_t)wall_clock64() : 0;
}

// A key's presence in a chunk index (launch_chunk_index: (key << 32) | (i + 1) per chunk, 0 = empty): every chunk
// with the key lies on the key's probe path before its first empty slot
__device__ __forceinline__ bool kslots_has(const unsigned long long* __restrict__ ks, uint32_t mask, uint32_t key) {
    uint32_t h = slot_hash(key) & mask;
    for (;;) {
        const unsigned long long v = ks[h];
        if (v == 0ull) return false;
        if ((uint32_t)(v >> 32) == key) return true;
        h = (h + 1) & mask;
    }
}

// The chain walk's key set: the table's distinct weak sums in LDS as a bucketed cuckoo set -- 2 x 8192 buckets of 2
// keys (128 KiB), a key in bucket h1(k) of the first half or h2(k) of the second.  A bucket's free slots hold its own
// empty value, a key that can never live in that bucket (its hashes point elsewhere), so every 32-bit key -- 0
// included -- is stored as itself, and a lookup is two 8-byte LDS reads and four compares, exact.  The hashes
// multiply 24-bit folds of the key by 24-bit constants (full-rate v_mul_u32_u24; a 32-bit multiply issues at quarter
// rate), a different fold per table, so that keys sharing one fold still part in the other table.  Config 4's 16384
// keys fill half of it; a key still displaced after the insertion's bound (tables near or above 32768 distinct keys,
// or keys crowding a few buckets) marks the set incomplete, and the walk then confirms every key in the chunk index.
constexpr int CHAIN_CK_BUCKETS = 8192;
__host__ __device__ constexpr uint32_t chain_ck_h1(uint32_t k) {
    return (((k ^ (k >> 15)) & 0xFFFFFFu) * 0x9E3779u) >> 19;
}
__host__ __device__ constexpr uint32_t chain_ck_h2(uint32_t k) {
    return CHAIN_CK_BUCKETS + ((((k ^ (k >> 8)) & 0xFFFFFFu) * 0x85EBCBu) >> 19);
}
// bucket i's empty value: 0, except in the two buckets key 0 hashes to, which use 1 (whose own buckets differ)
__host__ __device__ constexpr uint32_t chain_ck_empty(uint32_t i) {
    return (i == chain_ck_h1(0u) || i == chain_ck_h2(0u)) ? 1u : 0u;
}
static_assert(chain_ck_h1(1u) != chain_ck_h1(0u) && chain_ck_h2(1u) != chain_ck_h2(0u), "empty values");
struct ChainKeySet {
    uint2* b;       // 2 * CHAIN_CK_BUCKETS buckets
    int32_t* full;  // some key found no slot: lookups are not exact
};
__device__ __forceinline__ void chain_ck_insert(const ChainKeySet& ks, uint32_t k) {
    // cuckoo insertion: a free slot of the key's bucket in table w, else displace one of that bucket's keys and
    // carry it to its bucket in the other table (every key lives in its own h1 or h2 bucket; slots only ever go
    // from empty to a key)
    uint32_t cur = k;
    int w = 0;
    for (int it = 0; it < 128; ++it) {
        const uint32_t bi = w == 0 ? chain_ck_h1(cur) : chain_ck_h2(cur), e = chain_ck_empty(bi);
        uint32_t* slot = reinterpret_cast<uint32_t*>(&ks.b[bi]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t old = atomicCAS(slot + j, e, cur);
            if (old == e || old == cur) return;
        }
        const uint32_t old = atomicExch(slot + (it & 1), cur);
        if (old == cur) return;
        cur = old;
        w ^= 1;
    }
    *ks.full = 1;  // a key is left over: the set is not exact
}
__device__ __forceinline__ bool chain_ck_has(const ChainKeySet& ks, uint32_t k) {
    const uint2 a = ks.b[chain_ck_h1(k)], c = ks.b[chain_ck_h2(k)];
    return a.x == k || a.y == k || c.x == k || c.y == k;
}

// bit i: keys[i] is in the key set (exact sets only).  Branch free: two 8-byte reads and four compares per key (a
// wave's lanes would take every branch anyway)
__device__ __forceinline__ uint32_t chain_mask16(const ChainKeySet& set, const uint32_t (&keys)[16]) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t k = keys[i];
        const uint2 x = set.b[chain_ck_h1(k)], y = set.b[chain_ck_h2(k)];
        m |= (uint32_t)((x.x == k) | (x.y == k) | (y.x == k) | (y.y == k)) << i;
        if ((i & 3) == 3) asm volatile("" ::: "memory");  // 4 keys' reads in flight at a time (registers)
    }
    return m;
}

// The first of a lane's 16 keys (bit i of valid: position i is in the search) that the table holds, or -1: the 16
// first hash slots in one burst of independent loads (as probe_first_kernel: most keys are decided by their first
// slot, so a lane waits for about one L2 round trip, not 16), then the full lookup only for keys whose first slot
// holds another key, in order and only before the first certain hit (one out-of-line lookup loop, few registers)
__device__ __forceinline__ int chain_first_hit16(const unsigned long long* __restrict__ ks, uint32_t kmask,
                                                 const ChainKeySet& set, const uint32_t (&keys)[PROBE_PPT],
                                                 uint32_t valid) {
    // the key set in LDS: exact (the usual case), so the table in global memory is not touched at all
    if (*set.full == 0) {
        const uint32_t m = chain_mask16(set, keys) & valid;
        return m ? __builtin_ctz(m) : -1;
    }
    uint32_t hit = 0, need = 0;
    {
        unsigned long long sl[PROBE_PPT];
#pragma unroll
        for (int i = 0; i < PROBE_PPT; ++i) sl[i] = (valid >> i) & 1u ? ks[slot_hash(keys[i]) & kmask] : 0ull;
#pragma unroll
        for (int i = 0; i < PROBE_PPT; ++i) {
            if (sl[i] == 0ull) continue;
            if ((uint32_t)(sl[i] >> 32) == keys[i]) hit |= 1u << i;
            else need |= 1u << i;
        }
    }
    hit &= valid;
    need &= valid & (hit ? (hit & (0u - hit)) - 1u : 0xFFFFFFFFu);
    while (need) {
        const int i = __builtin_ctz(need);
        uint32_t kk = 0;
#pragma unroll
        for (int j = 0; j < PROBE_PPT; ++j)
            if (j == i) kk = keys[j];
        if (kslots_has(ks, kmask, kk)) return i;
        need &= need - 1u;
    }
    return hit ? __builtin_ctz(hit) : -1;
}

// An unaligned hit's window digest (MD5 of its L bytes, the seed appended, dl bytes kept), by the whole workgroup: the
// bytes staged through LDS in pieces of CHAIN_WIN_BUF, then compressed by one lane on the VALU.  One message is one
// dependent chain (~160 us for an 8 KiB window; a scalar-unit form measured slower: DESIGN.md section 5a).  Out of
// line, so that the walk's tile search keeps its registers.
constexpr int CHAIN_WIN_BUF = 16384;
// Stage piece [c0, c0 + len) of the window at x into buf (16-byte aligned source loads, byte stores that take the
// misalignment out; every granule overlaps the piece, so it lies in a page the source occupies) and, for the last
// piece, the seed, 0x80, zeros and the message's bit length (L + 4 bytes) to a whole block.  Returns the padded length.
__device__ __forceinline__ uint32_t chain_window_stage(const uint8_t* x, uint32_t L, uint32_t seed, uint8_t* buf,
                                                       uint32_t c0) {
    const int t = threadIdx.x;
    const uint32_t len = L - c0 < (uint32_t)CHAIN_WIN_BUF ? L - c0 : (uint32_t)CHAIN_WIN_BUF;
    const bool last = c0 + len == L;
    const uintptr_t xa = reinterpret_cast<uintptr_t>(x) + c0, a0 = xa & ~(uintptr_t)15;
    const int32_t shift = (int32_t)(xa - a0);
    for (int32_t g = 16 * t; g < shift + (int32_t)len; g += 16 * CHAIN_THREADS) {
        const uint4 q = *reinterpret_cast<const uint4*>(a0 + (uintptr_t)g);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int32_t o = g + k - shift;
            if (o >= 0 && o < (int32_t)len) buf[o] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        }
    }
    const uint32_t plen = last ? ((len + 4 + 1 + 8 + 63) & ~63u) : len;
    if (last && (uint32_t)t < plen - len) {
        const uint32_t i = len + (uint32_t)t;
        const uint64_t bits = ((uint64_t)L + 4) * 8;
        uint32_t v = 0;
        if (t < 4) v = (seed >> (8 * t)) & 0xFFu;
        else if (t == 4) v = 0x80u;
        else if (i >= plen - 8) v = (uint32_t)(bits >> (8 * (i - (plen - 8)))) & 0xFFu;
        buf[i] = (uint8_t)v;
    }
    __syncthreads();
    return plen;
}
// ... lane 0 compressing them on the VALU (md5_compress: v_bitop3 round functions), the words from LDS
__device__ __attribute__((noinline)) void chain_window_digest(const uint8_t* x, uint32_t L, uint32_t dl, uint32_t seed,
                                                              uint8_t* buf, uint8_t* dig) {
    const int t = threadIdx.x;
    Md5State st = md5_init();
    for (uint32_t c0 = 0; c0 < L; c0 += CHAIN_WIN_BUF) {
        const uint32_t plen = chain_window_stage(x, L, seed, buf, c0);
        if (t == 0) {
            const uint4* bq = reinterpret_cast<const uint4*>(buf);
            for (uint32_t b = 0; b < plen / 64; ++b) {
                uint32_t m[16];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint4 v = bq[4 * b + i];
                    m[4 * i] = v.x, m[4 * i + 1] = v.y, m[4 * i + 2] = v.z, m[4 * i + 3] = v.w;
                }
                md5_compress(st, m);
            }
        }
        __syncthreads();
    }
    if (t == 0) store_digest(dig, st, dl);
    __syncthreads();
}

// dl (1..16) digest bytes at a, packed four to a word, zero past dl: every byte's load issued before any use (one
// round trip, not dl), in as few loads as dl needs (4, 8 or 16; indices past dl re-read the last byte)
template <int NB>
__device__ __forceinline__ void chain_digest_load_n(const uint8_t* __restrict__ a, int dl, uint32_t (&w)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = 0u;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const uint32_t v = a[j < dl ? j : dl - 1];  // (unconditional: all NB loads go out together)
        w[j >> 2] |= (j < dl ? v : 0u) << (8 * (j & 3));
    }
}
__device__ __forceinline__ void chain_digest_load(const uint8_t* __restrict__ a, int dl, uint32_t (&w)[4]) {
    if (dl <= 4) chain_digest_load_n<4>(a, dl, w);
    else if (dl <= 8) chain_digest_load_n<8>(a, dl, w);
    else chain_digest_load_n<16>(a, dl, w);
}
// a digest already in registers (bytes packed four to a word, zero past dl) against dl bytes at b
__device__ __forceinline__ bool chain_digest_eq_reg(const uint32_t (&a)[4], const uint8_t* __restrict__ b, int dl) {
    uint32_t w[4];
    chain_digest_load(b, dl, w);
    return ((a[0] ^ w[0]) | (a[1] ^ w[1]) | (a[2] ^ w[2]) | (a[3] ^ w[3])) == 0u;
}
__device__ __forceinline__ bool chain_digest_eq(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int dl) {
    uint32_t w[4];
    chain_digest_load(a, dl, w);
    return chain_digest_eq_reg(w, b, dl);
}

// A wide tile lane's sums over its 32 positions' bytes x at p0 and y at p0 + B, weights relative to the tile start
// (base = p0 - q0): (sum x, sum (base + j) x, sum y, sum (base + B + j) y), j = 0..31 -- four bytes per v_dot4_i32_i8
// against the byte weights j (signed bytes, as Java's)
__device__ __forceinline__ void chain_lane_sums(const uint32_t (&xa)[2][4], const uint32_t (&xb)[2][4], uint32_t base,
                                                uint32_t B, int32_t (&pre)[4]) {
    int32_t sa = 0, ja = 0, sb = 0, jb = 0;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int wt = 0x03020100 + 0x04040404 * d + 0x10101010 * hh;  // bytes 16 hh + 4 d + 0..3
            sa = __builtin_amdgcn_sdot4((int)xa[hh][d], 0x01010101, sa, false);
            ja = __builtin_amdgcn_sdot4((int)xa[hh][d], wt, ja, false);
            sb = __builtin_amdgcn_sdot4((int)xb[hh][d], 0x01010101, sb, false);
            jb = __builtin_amdgcn_sdot4((int)xb[hh][d], wt, jb, false);
        }
    pre[0] = sa;
    pre[1] = (int32_t)(base * (uint32_t)sa) + ja;
    pre[2] = sb;
    pre[3] = (int32_t)((base + B) * (uint32_t)sb) + jb;
}

// the table's distinct weak sums into the workgroup's key set
__device__ __forceinline__ void chain_kset_build(const ChainKeySet& ks, const int32_t* __restrict__ weak, int64_t C) {
    const int t = threadIdx.x;
    for (int i = t; i < 2 * CHAIN_CK_BUCKETS; i += CHAIN_THREADS) {
        const uint32_t e = chain_ck_empty((uint32_t)i);
        ks.b[i] = make_uint2(e, e);
    }
    if (t == 0) *ks.full = 0;
    __syncthreads();
    for (int64_t c = t; c < C; c += CHAIN_THREADS) chain_ck_insert(ks, (uint32_t)weak[c]);
    __syncthreads();
}

// the map's shared words: relaxed atomics at agent scope (the workgroups sit on different XCDs, whose L2s are not
// coherent with each other); vector memory operations throughout
__device__ __forceinline__ int32_t chain_ld(const int32_t* p) {
    return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t chain_ld64(const int64_t* p) {
    return __hip_atomic_load(const_cast<int64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void chain_st(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void chain_st64(int64_t* p, int64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One tile of a file's hit map: positions [q0, q0 + CHAIN_TILE) below hend, q0 a multiple of CHAIN_TILE.  The keys
// are the walk's wide-tile keys in the synced state (each lane anchored on its block's aligned sum T(o), the prefix
// sums from one exscan rebased at each block's first lane, the head of the block the tile starts in); bit i of
// lane t's word = position q0 + 32 t + i hits the key set.  Stored as (gen << 32) | bits, one 8-byte store.
__device__ void chain_map_tile(const ChainFile& F, int64_t q0, uint32_t gen, const ChainKeySet& kset, int32_t* sh,
                               int32_t (*s_seg)[4]) {
    const int t = threadIdx.x;
    const int64_t n = F.n, B = F.B, hend = F.hend;
    const int64_t kb0 = q0 / B, o0 = kb0 * B;
    int32_t head[4] = {0, 0, 0, 0};
    if (q0 > o0) {
        range_sums(F.data, n, o0, q0, o0, head[0], head[1]);
        range_sums(F.data, n, o0 + B, q0 + B, o0, head[2], head[3]);
        block_reduce<4>(head, sh);
    }
    const int64_t p0 = q0 + (int64_t)t * CHAIN_PPT;
    const int64_t kb = p0 / B, o = kb * B;
    uint32_t xa[2][4], xb[2][4];
    load16(F.data, n, p0, xa[0]);
    load16(F.data, n, p0 + 16, xa[1]);
    load16(F.data, n, p0 + B, xb[0]);
    load16(F.data, n, p0 + B + 16, xb[1]);
    const bool live = p0 < hend;
    const int32_t To = live ? F.aw[kb] : 0;
    int32_t pre[4];
    chain_lane_sums(xa, xb, (uint32_t)(p0 - q0), (uint32_t)B, pre);
    block_exscan<4>(pre, sh);
    if (p0 == o) {
#pragma unroll
        for (int v = 0; v < 4; ++v) s_seg[kb - kb0][v] = pre[v];
    }
    __syncthreads();
    if (live) {
        uint32_t pa, pa2, pb, pb2;
        if (o < q0) {
            const uint32_t d = (uint32_t)(q0 - o);
            pa = (uint32_t)head[0] + (uint32_t)pre[0];
            pa2 = (uint32_t)head[1] + (uint32_t)pre[1] + d * (uint32_t)pre[0];
            pb = (uint32_t)head[2] + (uint32_t)pre[2];
            pb2 = (uint32_t)head[3] + (uint32_t)pre[3] + d * (uint32_t)pre[2];
        } else {
            const int32_t* L = s_seg[kb - kb0];
            const uint32_t d = (uint32_t)(o - q0);
            pa = (uint32_t)(pre[0] - L[0]);
            pa2 = (uint32_t)(pre[1] - L[1]) - d * pa;
            pb = (uint32_t)(pre[2] - L[2]);
            pb2 = (uint32_t)(pre[3] - L[3]) - d * pb;
        }
        const uint32_t s1o = (uint32_t)To & 0xFFFFu, s2o = (uint32_t)To >> 16;
        const uint32_t P1e = s1o + pb;
        const uint32_t P2e = (uint32_t)B * s1o - s2o + pb2;
        uint32_t u1 = P1e - pa;
        uint32_t u2 = (uint32_t)(p0 + B - o) * u1 - (P2e - pa2);
        uint32_t bits = 0;
#pragma unroll 1
        for (int hh = 0; hh < 2; ++hh) {
            uint32_t wa[4], wb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                wa[j] = hh ? xa[1][j] : xa[0][j];
                wb[j] = hh ? xb[1][j] : xb[0][j];
            }
            uint32_t keys[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                keys[i] = (u1 & 0xFFFFu) | (u2 << 16);
                const int32_t xo = sbyte_of(wa, i), xi = sbyte_of(wb, i);
                u1 += (uint32_t)(xi - xo);
                u2 += u1 - (uint32_t)__mul24((int)B, xo);  // (B <= 2^17: a full-rate 24-bit multiply)
            }
            bits |= chain_mask16(kset, keys) << (16 * hh);
        }
        if (hend - p0 < 32) bits &= (1u << (uint32_t)(hend - p0)) - 1u;  // windows past hend: not searched
        __hip_atomic_store(&F.hmap[p0 >> 5], ((unsigned long long)gen << 32) | bits, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // (s_seg and sh: the next tile)
}

constexpr int CHAIN_HELP_LEAD = 64;   // a helper stays with its file while the map leads the walk by fewer segments
// A helper workgroup: while some walk that has searched ChainHelp::help_tiles tiles is still running, take the next
// unmapped segment of the one whose map leads it least (its own current file while the lead is short: the key set is
// built per file) -- never the segment the walk is in, which it will finish first -- and map it tile by tile,
// stopping when the walk ends or has passed the tile.  While walks are running that have not searched that far yet it
// sleeps and looks again; once no mappable walk is running it leaves.  No walk ever waits for a helper: a walk reads
// a map word only when it carries this launch's generation, and searches the tile itself otherwise.  (A helper waits
// only for walks of its own launch, whose workgroups precede it in dispatch order.)
__device__ __attribute__((noinline)) void chain_help(const ChainFile* __restrict__ files, int nfiles, uint32_t gen,
                                                     ChainHelp* help, uint2* ck, int32_t* ck_full,
                                                     int32_t* sh, int32_t (*s_seg)[4], unsigned long long* s_best,
                                                     int32_t* s_word, int32_t* s_live, bool timed) {
    const int t = threadIdx.x;
    const ChainKeySet kset{ck, ck_full};
    int cur = -1;
    ChainFile F = files[0];
    for (;;) {
        if (t == 0) {
            *s_best = 0ull;
            *s_live = 0;
        }
        __syncthreads();
        for (int f = t; f < nfiles; f += CHAIN_THREADS) {
            ChainHelp* h = help + f;
            const int32_t nseg = h->nseg;  // (written by the host before the launch)
            if (nseg == 0) continue;
            // one round trip for the file's shared words
            const int32_t live = chain_ld(&h->live), tiles = chain_ld(&h->tiles), claim = chain_ld(&h->claim);
            const int32_t nhelp = chain_ld(&h->nhelp);
            const int64_t pos = chain_ld64(&h->pos);
            if (live == 0 || claim >= nseg) continue;
            *s_live = 1;  // a walk that may still search: wait for it rather than leave
            if (tiles < h->help_tiles) continue;
            // the most urgent files first -- the map's frontier least far ahead of the walk, in four levels -- then
            // the fewest helpers, then a hash that spreads the helpers; the current file while the map leads its
            // walk by fewer than CHAIN_HELP_LEAD segments (its key set is built)
            const int64_t lead = (int64_t)claim - pos / CHAIN_MAP_SEG;
            const uint32_t level = lead <= 0 ? 3u : lead <= 4 ? 2u : lead <= 16 ? 1u : 0u;
            const uint32_t few = 255u - (uint32_t)(nhelp < 0 ? 0 : nhelp > 255 ? 255 : nhelp);
            const uint32_t tie = ((uint32_t)f * 0x9E3779B1u) ^ ((uint32_t)blockIdx.x * 0x85EBCA77u);
            const unsigned long long key = ((unsigned long long)(f == cur && lead < CHAIN_HELP_LEAD) << 63) |
                                           ((unsigned long long)level << 61) | ((unsigned long long)few << 53) |
                                           ((unsigned long long)(tie >> 1) << 21) | (uint32_t)f;
            atomicMax(s_best, key);
        }
        __syncthreads();
        const unsigned long long best = *s_best;
        const bool any_live = *s_live != 0;
        __syncthreads();
        if (best == 0ull) {
            if (!any_live) break;  // every mappable walk has ended: nothing will come
            __builtin_amdgcn_s_sleep(64);  // walks still short of their help_tiles: look again shortly
            continue;
        }
        const int f = (int)(best & 0xFFFFFull);
        ChainHelp* h = help + f;
        if (t == 0) {  // the segment the walk is in and those behind it are skipped, not claimed one by one
            atomicMax(&h->claim, (int32_t)(chain_ld64(&h->pos) / CHAIN_MAP_SEG) + 1);
            *s_word = atomicAdd(&h->claim, 1);
        }
        __syncthreads();
        const int32_t seg = *s_word;
        __syncthreads();
        if (seg >= h->nseg) continue;
        if (f != cur) {
            if (t == 0) {
                if (cur >= 0) atomicSub(&help[cur].nhelp, 1);
                atomicAdd(&h->nhelp, 1);
            }
            cur = f;
            const int64_t tb = chain_clock(timed);
            F = files[f];
            chain_kset_build(kset, F.table_weak, F.C);
            if (t == 0) {
                atomicAdd((unsigned long long*)&h->t_kset, (unsigned long long)(chain_clock(timed) - tb));
                atomicAdd(&h->joins, 1);
            }
            if (*kset.full) {  // not exact: the walk confirms keys in the chunk index; no map for this file
                if (t == 0) atomicMax(&h->claim, h->nseg);
                __syncthreads();
                continue;
            }
        }
        const int64_t lo = (int64_t)seg * CHAIN_MAP_SEG, hi = lo + CHAIN_MAP_SEG < F.hend ? lo + CHAIN_MAP_SEG : F.hend;
        bool whole = true;
        for (int64_t q0 = lo; q0 < hi; q0 += CHAIN_TILE) {
            if (t == 0) *s_word = chain_ld(&h->live) != 0 && chain_ld64(&h->pos) < q0 + CHAIN_TILE;
            __syncthreads();
            const bool go = *s_word != 0;
            __syncthreads();
            if (!go) {
                whole = false;
                break;
            }
            chain_map_tile(F, q0, gen, kset, sh, s_seg);
        }
        if (t == 0) {
            atomicAdd(&h->mapped, 1);
            if (whole) {
                atomicAdd(&h->whole, 1);
                atomicMin((unsigned long long*)&h->t_first, (unsigned long long)chain_clock(timed));
            }
        }
    }
    if (t == 0 && cur >= 0) atomicSub(&help[cur].nhelp, 1);
}

__global__ __launch_bounds__(CHAIN_THREADS) void chain_advance_kernel(const ChainFile* __restrict__ files, int phase,
                                                                      int abort_gen, ChainHelp* help, int nfiles,
                                                                      int timed) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[4 * CHAIN_THREADS / 64];
    __shared__ int32_t s_hit;                  // first hit in a tile (offset from the tile start), or INT_MAX
    __shared__ uint32_t s_key;                 // its key
    __shared__ int32_t s_sc[4];                // an aligned map hit's own chunk: flag && !dup, then the next step's words
    __shared__ int32_t s_bk[CHAIN_BUCKET_CAP];  // bucket of the key (ascending chunk index)
    __shared__ int32_t s_nbk;
    __shared__ int64_t s_zero;                 // first unset chain flag
    __shared__ __attribute__((aligned(16))) uint8_t s_win[CHAIN_WIN_BUF + 128];  // an unaligned window's bytes (its digest: s_dig)
    __shared__ int32_t s_any;                  // some chunk carries the stale digest
    __shared__ int32_t s_seg[CHAIN_SEGS][4];   // wide tiles: the exscan at each block's first lane
    __shared__ uint2 s_ck[2 * CHAIN_CK_BUCKETS];  // the table's keys (ChainKeySet)
    __shared__ int32_t s_ck_full;
    __shared__ __attribute__((aligned(16))) uint8_t s_dig[16];
    __shared__ rsh_event s_ev[CHAIN_EV_LDS];   // finished events not yet in F.ev
    __shared__ unsigned long long s_best;      // helpers: the file to map next
    __shared__ int32_t s_word, s_live;
    const ChainKeySet kset{s_ck, &s_ck_full};
    if ((int)blockIdx.x >= nfiles) {  // a helper workgroup (phase 0): it only maps
        chain_help(files, nfiles, (uint32_t)abort_gen, help, s_ck, &s_ck_full, sh, s_seg, &s_best, &s_word, &s_live,
                   timed != 0);
        return;
    }
    // the descriptor by value: it sits in pinned host memory, and a reference would let the compiler re-read its
    // fields across the loop (the event stores may alias it) -- a PCIe round trip each
    const ChainFile F = files[blockIdx.x];
    ChainHelp* const H = (phase == 0 && help != nullptr) ? help + blockIdx.x : nullptr;
    if (H != nullptr && threadIdx.x == 0) chain_st64(&H->t_start, chain_clock(timed));
    const uint32_t map_gen = (H != nullptr && F.hmap != nullptr) ? (uint32_t)abort_gen : 0u;  // 0: no map
    ChainOut* out = F.out;
    // phase 0 walks over the prefix speculation [0, na_a); phase 1 resumes the walks that reached its end
    if (phase == 1 && out->status != CHAIN_MORE) return;
    const int t = threadIdx.x;
    const int64_t n = F.n, B = F.B, C = F.C;
    const int dl = F.dl;
    const int64_t S = F.rem > 0 ? F.rem : B;  // Checksum.java:131-137
    const int64_t last = n - S, nB = n - B;
    const int64_t na = phase == 0 ? F.na_a : F.na, nflags = na < C ? na : C;
    const bool wide = (B % CHAIN_PPT) == 0 && B >= 512 && CHAIN_TILE / B + 2 <= CHAIN_SEGS;
    int64_t s = out->s, m = out->m;
    // The key set (~C LDS inserts, tens of microseconds) only if the walk may search: a walk that starts aligned on
    // an unbroken run of chain flags up to the last window with a chunk (an identical file, or its rest after the
    // prefix) follows the chain and never looks a key up; should it need one after all, it stops there (the host).
    bool kset_built = true;
    if (s % B == 0 && nflags >= na) {
        if (t == 0) s_zero = nflags;
        __syncthreads();
        // one 16-byte line of flags per lane per pass (as in step (1) below), masked to [s / B, nflags)
        const int64_t k = s / B;
        const uintptr_t fa = reinterpret_cast<uintptr_t>(F.flags);
        for (uintptr_t l0 = (fa + (uintptr_t)k) & ~(uintptr_t)15; l0 < fa + (uintptr_t)nflags;
             l0 += 16u * CHAIN_THREADS) {
            const uintptr_t la = l0 + 16u * (uintptr_t)t;
            const int64_t jb = (int64_t)la - (int64_t)fa;
            if (la < fa + (uintptr_t)nflags) {
                uint32_t w[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
                if (la + 16 <= fa + (uintptr_t)nflags) {
                    const uint4 q = *reinterpret_cast<const uint4*>(la);
                    w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
                } else {
                    for (int i = 0; i < 16; ++i)
                        if (jb + i >= 0 && jb + i < nflags && F.flags[jb + i] == 0) w[i >> 2] &= ~(0xFFu << (8 * (i & 3)));
                }
                int64_t z = -1;
#pragma unroll
                for (int i = 15; i >= 0; --i)
                    if (jb + i >= k && jb + i < nflags && ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == 0u) z = jb + i;
                if (z >= 0) atomicMin((unsigned long long*)&s_zero, (unsigned long long)z);
            }
        }
        __syncthreads();
        kset_built = s_zero < nflags;  // (uniform) a break in the chain: the walk will search
        __syncthreads();
    }
    const int64_t tks0 = chain_clock(timed);
    if (kset_built) chain_kset_build(kset, F.table_weak, C);
    const int64_t t_kset = chain_clock(timed) - tks0;
    int32_t pref = out->pref;
    int32_t nev = out->n_ev, status = CHAIN_STOP;
    int64_t lit = out->literal, mat = out->matched, chain_matches = out->chain_matches, events = out->events;
    int32_t tiles = out->tiles, digests = out->digests, poisoned = 0, dead = 0, mapped = out->mapped;
    int32_t first_mapped = out->first_mapped;
    int64_t flushes = out->flushes;
    const int64_t tk0 = chain_clock(timed);
    int64_t t_tiles = 0, t_check = 0, t_event = 0, t_digest = 0, t_chain = 0, t_drain = 0, t_evb = 0;
    const uint8_t* stale = nullptr;  // poisoned: the cached digest
    uint32_t dg[4] = {0u, 0u, 0u, 0u};  // the window's digest at the current event (poisoned: the stale one)
    int64_t clear_to = -1;            // stopped at a flush point: no candidate in [s, clear_to]
    int32_t why = CHAIN_WHY_NONE;
    uint32_t desync_lo = 0, desync_hi = 0;  // CHAIN_WHY_FLUSHED: E at s after the walk's flush
    // the loop's first words for the step at pf_s with preferred index pf_pref, loaded by the event before it
    int64_t pf_s = -1;
    int32_t pf_pref = -1, pf_aw = 0, pf_tw = 0;
    uint8_t pf_flag = 0;
    rsh_event pend{0, 0, 0, 0, 0, 0};  // the event being built (lane 0 writes it when the next one starts)
    bool have = false;
    if (nev > 0) {  // phase 1: the last event stays open (a MATCH run may go on across the prefix's end)
        pend = F.ev[nev - 1];
        have = true;
        --nev;
    }
    // Finished events collect in LDS and go to the event buffer (pinned host memory) CHAIN_EV_LDS at a time, one per
    // thread: a store to host memory is a PCIe write whose completion the next vmcnt wait of its wave waits for (on
    // gfx9 the counter covers stores too), so lane 0 writing each event itself held the walk ~1-2 us per event.
    int32_t nev_w = nev;  // events already in F.ev
    auto drain_ev = [&]() {  // (all threads)
        const int64_t tdr0 = chain_clock(timed);
        __syncthreads();
        for (int32_t i = t; i < nev - nev_w; i += CHAIN_THREADS) F.ev[nev_w + i] = s_ev[i];
        nev_w = nev;
        __syncthreads();
        t_drain += chain_clock(timed) - tdr0;
    };
    auto flush_pend = [&]() {  // (the loop drains at its top while fewer than CHAIN_EV_LDS - 8 are held)
        if (have) {
            if (t == 0) s_ev[nev - nev_w] = pend;
            ++nev;
        }
        have = false;
    };
    auto emit_lit = [&](int64_t off, int64_t len) {  // Sender.sendDataFrom; zero-length calls write nothing
        if (len <= 0) return;
        flush_pend();
        pend = rsh_event{off, len, RSH_EV_LITERAL, 0, 0, 0};
        have = true;
        lit += len;
    };
    auto emit_match = [&](int64_t off, int64_t len, int32_t idx, int32_t cnt) {
        mat += len;
        if (have && pend.kind == RSH_EV_MATCH && pend.index + pend.count == idx && pend.offset + pend.length == off) {
            pend.count += cnt;
            pend.length += len;
            return;
        }
        flush_pend();
        pend = rsh_event{off, len, RSH_EV_MATCH, idx, cnt, 0};
        have = true;
    };

    for (;;) {
        if (nev - nev_w >= CHAIN_EV_LDS - 8) drain_ev();  // (a step adds at most three)
        if (nev + 3 > F.ev_cap) {  // room for a pending event, a literal and a match
            why = CHAIN_WHY_EVCAP;
            break;
        }
        if (s > last) {  // the loop ends (Sender.java:1313-1316)
            emit_lit(m, n - m);
            status = CHAIN_DONE;
            why = CHAIN_WHY_END;
            break;
        }
        // phase-shifted windows: the host's phase speculation.  A poisoned walk (a stale cached digest, quirk B) goes
        // on from any position: only step (2) applies to it, and every candidate is compared with the stale digest
        if (s % B != 0 && !poisoned) {
            why = CHAIN_WHY_PHASE;
            break;
        }
        const int64_t k = s / B;
        const bool al = s % B == 0;
        // the words steps (1), (1') and (2) look at first, loaded together: one global round trip per step instead of
        // three in sequence (a desynced walk takes these steps once per event)
        // (or loaded already: an aligned event's match is usually its own chunk kp, and the event then issued the
        // next step's words beside its bucket and digests -- see below)
        const bool pf_use = pf_s == s && pf_pref == pref && !poisoned;
        const uint8_t flag_k = pf_use ? pf_flag : (!poisoned && k == pref && k < nflags) ? F.flags[k] : (uint8_t)0;
        const int32_t aw_k = pf_use ? pf_aw : (al && k < na) ? F.aw[k] : 0;
        const int32_t tw_pref = pf_use ? pf_tw : (!poisoned && pref < C && k < na) ? F.table_weak[pref] : 0;
        pf_s = -1;
        // (1) aligned chain: preferred index == k and source window k carries chunk k's sums
        const int64_t tch0 = chain_clock(timed);
        if (flag_k) {
            if (t == 0) s_zero = nflags;
            __syncthreads();
            // one aligned 16-byte line of flags per lane per pass: an identical file's 16384 flags in two passes
            // instead of 32 load-and-barrier rounds.  A line may start before flag k (or before the file's flags,
            // inside the batch's flag buffer) and is masked to [k, nflags); a line past the end is read bytewise.
            const uintptr_t fa = reinterpret_cast<uintptr_t>(F.flags);
            for (uintptr_t l0 = (fa + (uintptr_t)k) & ~(uintptr_t)15; l0 < fa + (uintptr_t)nflags;
                 l0 += 16u * CHAIN_THREADS) {
                const uintptr_t la = l0 + 16u * (uintptr_t)t;
                const int64_t jb = (int64_t)la - (int64_t)fa;  // flag index of the line's first byte
                int64_t z = -1;
                if (la < fa + (uintptr_t)nflags) {
                    uint32_t w[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
                    if (la + 16 <= fa + (uintptr_t)nflags) {
                        const uint4 q = *reinterpret_cast<const uint4*>(la);
                        w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
                    } else {
                        for (int i = 0; i < 16; ++i)
                            if (jb + i >= 0 && jb + i < nflags && F.flags[jb + i] == 0) w[i >> 2] &= ~(0xFFu << (8 * (i & 3)));
                    }
#pragma unroll
                    for (int i = 15; i >= 0; --i)
                        if (jb + i >= k && jb + i < nflags && ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == 0u) z = jb + i;
                }
                if (z >= 0) atomicMin((unsigned long long*)&s_zero, (unsigned long long)z);
                __syncthreads();
                if (s_zero < nflags) break;
            }
            const int64_t j_end = s_zero;
            __syncthreads();
            const int64_t t_max = (last - s) / B + 1;
            const int64_t tt = (j_end - k < t_max) ? j_end - k : t_max;
            const int64_t j = k + tt, p = (s + tt * B < n) ? s + tt * B : n;
            emit_lit(m, s - m);
            emit_match(s, p - s, (int32_t)k, (int32_t)(j - k));
            chain_matches += j - k;
            s = m = p;
            pref = (int32_t)j;
            t_chain += chain_clock(timed) - tch0;
            continue;
        }
        // (1') the window at s against chunk pref while both sums agree (windows s + iB, chunks pref + i)
        if (!poisoned && pref < C && k < na) {
            int64_t lim = na - k;
            if (C - pref < lim) lim = C - pref;
            if ((last - s) / B + 1 < lim) lim = (last - s) / B + 1;
            int64_t tt = 0;
            if (lim > 0 && aw_k == tw_pref && chain_digest_eq(F.as + k * dl, F.table_strong + (int64_t)pref * dl, dl)) {
                tt = 1;
                while (tt < lim && F.aw[k + tt] == F.table_weak[pref + tt] &&
                       chain_digest_eq(F.as + (k + tt) * dl, F.table_strong + (pref + tt) * dl, dl))
                    ++tt;
            }
            if (tt > 0) {
                const int64_t p = (s + tt * B < n) ? s + tt * B : n;
                emit_lit(m, s - m);
                emit_match(s, p - s, pref, (int32_t)tt);
                s = m = p;
                pref += (int32_t)tt;
                t_chain += chain_clock(timed) - tch0;
                continue;
            }
        }
        t_chain += chain_clock(timed) - tch0;
        // (2) the next candidate event in [s, stop]
        const int64_t f = (m + 10 * B <= n) ? m + 9 * B : INT64_MAX;
        const int64_t stop = f < last ? f : last;
        if (stop > nB) {  // shrinking windows near the end: the host
            why = CHAIN_WHY_TAIL;
            break;
        }
        // (see above: an unbroken chain needed no key set; should this step look a key up after all, the host takes
        // it -- at the prefix's end the search is empty and the walk goes on to its cut, as with a key set)
        if (!kset_built && (s / B < na || s <= (stop < na * B - 1 ? stop : na * B - 1))) {
            why = CHAIN_WHY_NOKSET;
            break;
        }
        int64_t p = -1;
        uint32_t key = 0;
        int64_t a = s;
        if (al && k < na) {
            key = (uint32_t)aw_k;
            if (s_ck_full ? kslots_has(F.kslots, F.kmask, key) : chain_ck_has(kset, key)) p = s;
            else a = s + 1;
        }
        bool sc_hit = false;  // the hit came from the map at an aligned window: s_sc holds its chunk's words
        bool cut = false;  // the search reached windows past the speculation (no anchor T(o))
        if (wide) {
            // tiles of CHAIN_TILE positions from a (lane-aligned), across block boundaries: each lane anchors its
            // 16 positions on its own block's T(o); the prefix sums from o come from one exscan over the tile
            // with weights relative to the tile start, rebased at each block's first lane (a segmented scan), and
            // the head of the block the tile starts in (range_sums from o to the tile)
            const int64_t lim_spec = na * B - 1;  // windows with an anchor: blocks < na
            const int64_t qlast = stop < lim_spec ? stop : lim_spec;
            if (H != nullptr && t == 0) {  // for the helpers: where this search starts, how many tiles so far
                chain_st64(&H->pos, a);
                chain_st(&H->tiles, tiles);
            }
            for (int64_t q0 = a & ~(int64_t)(CHAIN_PPT - 1); p < 0 && q0 <= qlast;) {
                ++tiles;
                const int64_t tt0 = chain_clock(timed);
                if (map_gen != 0u) {
                    // the tile from the hit map when every word it needs carries this launch's generation: lane t's
                    // word holds positions [q0 + 32 t, + 32), masked to [a, qlast] (qlast < hend)
                    const int64_t pm = q0 + (int64_t)t * CHAIN_PPT;
                    const int64_t lo = a > pm ? a - pm : 0, hi = qlast - pm;
                    const bool need = lo <= 31 && hi >= lo;
                    unsigned long long wv = 0ull;
                    if (need) wv = __hip_atomic_load(&F.hmap[pm >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    // beside it, the speculation's sum of an aligned window in the lane's range: a hit there needs
                    // no second round trip for its key
                    const bool al_lane = need && pm % B == 0;  // (pm <= qlast < na B)
                    const int32_t awl = al_lane ? F.aw[pm / B] : 0;
                    // ... and its chunk's chain flag and uniqueness with the next step's first words: an aligned hit
                    // on its own chunk (flag set) whose weak sum no other chunk has is decided without the bucket
                    const int64_t kl = pm / B, kl1 = kl + 1;
                    int32_t scw[4] = {0, 0, 0, 0};
                    if (al_lane && kl < nflags && kl < C) {
                        scw[0] = (F.flags[kl] != 0 && F.dup[kl] == 0) ? 1 : 0;
                        scw[1] = kl1 < nflags ? F.flags[kl1] : 0;
                        scw[2] = kl1 < na ? F.aw[kl1] : 0;
                        scw[3] = (kl1 < C && kl1 < na) ? F.table_weak[kl1] : 0;
                    }
                    if (t == 0) s_hit = 0x7FFFFFFF;
                    if (__syncthreads_and(!need || (uint32_t)(wv >> 32) == map_gen)) {
                        if (need) {
                            const uint32_t bits = (uint32_t)wv & (0xFFFFFFFFu >> (31 - (hi < 31 ? hi : 31))) &
                                                  (0xFFFFFFFFu << lo);
                            if (bits) atomicMin(&s_hit, (int32_t)(pm - q0) + __builtin_ctz(bits));
                        }
                        __syncthreads();
                        const int32_t hoff = s_hit;
                        if (hoff != 0x7FFFFFFF && al_lane && pm == q0 + hoff) {
                            s_key = (uint32_t)awl;
#pragma unroll
                            for (int v = 0; v < 4; ++v) s_sc[v] = scw[v];
                        }
                        __syncthreads();
                        if (hoff != 0x7FFFFFFF) {  // the key: the window's true weak sum (synced)
                            p = q0 + hoff;
                            if (p % B == 0) {      // an aligned window: the speculation's sum, loaded above
                                key = s_key;
                                sc_hit = true;
                            } else {               // else one reduction over its B bytes
                                int32_t w2[2] = {0, 0};
                                range_sums(F.data, n, p, p + B, p, w2[0], w2[1]);
                                block_reduce<2>(w2, sh);
                                const uint32_t S1 = (uint32_t)w2[0], S2 = (uint32_t)B * S1 - (uint32_t)w2[1];
                                key = (S1 & 0xFFFFu) | (S2 << 16);
                            }
                        }
                        if (mapped++ == 0) first_mapped = tiles;
                        q0 += CHAIN_TILE;
                        t_tiles += chain_clock(timed) - tt0;
                        continue;
                    }
                }
                const int64_t kb0 = q0 / B, o0 = kb0 * B;
                int32_t head[4] = {0, 0, 0, 0};
                if (q0 > o0) {
                    range_sums(F.data, n, o0, q0, o0, head[0], head[1]);
                    range_sums(F.data, n, o0 + B, q0 + B, o0, head[2], head[3]);
                    block_reduce<4>(head, sh);
                }
                const int64_t p0 = q0 + (int64_t)t * CHAIN_PPT;
                const int64_t kb = p0 / B, o = kb * B;
                uint32_t xa[2][4], xb[2][4];
                load16(F.data, n, p0, xa[0]);
                load16(F.data, n, p0 + 16, xa[1]);
                load16(F.data, n, p0 + B, xb[0]);
                load16(F.data, n, p0 + B + 16, xb[1]);
                const bool live = p0 <= stop && p0 <= lim_spec && p0 + CHAIN_PPT > a;
                const int32_t To = live ? F.aw[kb] : 0;
                int32_t pre[4];
                chain_lane_sums(xa, xb, (uint32_t)(p0 - q0), (uint32_t)B, pre);
                block_exscan<4>(pre, sh);  // sums over [q0, p0) and [q0 + B, p0 + B), weights j - q0
                if (p0 == o) {              // a block's first lane: its rebasing point
#pragma unroll
                    for (int v = 0; v < 4; ++v) s_seg[kb - kb0][v] = pre[v];
                }
                if (t == 0) s_hit = 0x7FFFFFFF;
                __syncthreads();
                const int64_t tc0 = chain_clock(timed);
                int32_t my_hit = 0x7FFFFFFF;
                uint32_t my_key = 0;
                if (live) {
                    uint32_t pa, pa2, pb, pb2;  // sums over [o, p0) and [o + B, p0 + B), weights j - o
                    if (o < q0) {               // the tile's first block: its head + the tile's part
                        const uint32_t d = (uint32_t)(q0 - o);
                        pa = (uint32_t)head[0] + (uint32_t)pre[0];
                        pa2 = (uint32_t)head[1] + (uint32_t)pre[1] + d * (uint32_t)pre[0];
                        pb = (uint32_t)head[2] + (uint32_t)pre[2];
                        pb2 = (uint32_t)head[3] + (uint32_t)pre[3] + d * (uint32_t)pre[2];
                    } else {                    // rebased at the block's first lane
                        const int32_t* L = s_seg[kb - kb0];
                        const uint32_t d = (uint32_t)(o - q0);
                        pa = (uint32_t)(pre[0] - L[0]);
                        pa2 = (uint32_t)(pre[1] - L[1]) - d * pa;
                        pb = (uint32_t)(pre[2] - L[2]);
                        pb2 = (uint32_t)(pre[3] - L[3]) - d * pb;
                    }
                    const uint32_t s1o = (uint32_t)To & 0xFFFFu, s2o = (uint32_t)To >> 16;
                    const uint32_t P1e = s1o + pb;
                    const uint32_t P2e = (uint32_t)B * s1o - s2o + pb2;
                    const uint32_t s1 = P1e - pa;
                    const uint32_t s2 = (uint32_t)(p0 + B - o) * s1 - (P2e - pa2);
                    // the lane's 32 positions as two halves of 16 (the first hit of the first half wins).  The two
                    // 16-bit halves of the rolling value are kept apart (u1, u2: each exact mod 2^16, the Java
                    // subtract-then-add of Rolling.java:25-60 in two adds each), packed into the key per position
                    uint32_t u1 = s1, u2 = s2;
                    const int64_t lim_p = stop < lim_spec ? stop : lim_spec;
#pragma unroll 1
                    for (int hh = 0; hh < 2; ++hh) {  // (not unrolled: one half's keys in registers at a time)
                        uint32_t wa[4], wb[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            wa[j] = hh ? xa[1][j] : xa[0][j];
                            wb[j] = hh ? xb[1][j] : xb[0][j];
                        }
                        uint32_t keys[16];
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            keys[i] = (u1 & 0xFFFFu) | (u2 << 16);
                            const int32_t xo = sbyte_of(wa, i), xi = sbyte_of(wb, i);
                            u1 += (uint32_t)(xi - xo);
                            u2 += u1 - (uint32_t)__mul24((int)B, xo);  // (B <= 2^17: a full-rate 24-bit multiply)
                        }
                        // positions base + i with a <= position <= lim_p, as a bit range
                        const int64_t base = p0 + 16 * hh;
                        const int64_t lo = a > base ? a - base : 0, hi = lim_p - base;
                        uint32_t valid = 0;
                        if (lo <= 15 && hi >= 0 && hi >= lo)
                            valid = (0xFFFFu >> (15 - (hi < 15 ? hi : 15))) & (0xFFFFu << lo);
                        if (my_hit == 0x7FFFFFFF) {
                            const int h = chain_first_hit16(F.kslots, F.kmask, kset, keys, valid);
                            if (h >= 0) {
                                my_hit = (int32_t)(p0 + 16 * hh + h - q0);
#pragma unroll
                                for (int i = 0; i < 16; ++i)  // (a static index: keys stays in registers)
                                    if (i == h) my_key = keys[i];
                            }
                        }
                    }
                    if (my_hit != 0x7FFFFFFF) atomicMin(&s_hit, my_hit);
                }
                __syncthreads();
                t_check += chain_clock(timed) - tc0;
                if (my_hit != 0x7FFFFFFF && my_hit == s_hit) s_key = my_key;
                __syncthreads();
                if (s_hit != 0x7FFFFFFF) {
                    p = q0 + s_hit;
                    key = s_key;
                }
                __syncthreads();
                q0 += CHAIN_TILE;
                t_tiles += chain_clock(timed) - tt0;
            }
            cut = p < 0 && stop > lim_spec;  // (lim_spec, stop] has no anchors: not searched
        }
        // narrow blocks (B not a multiple of 16, or < 512): tiles of PROBE_TILE positions in block coordinates
        for (int64_t q0 = (a / B) * B + ((a % B) / PROBE_TILE) * PROBE_TILE; !wide && p < 0 && q0 <= stop;) {
            const int64_t kb = q0 / B, o = kb * B;
            if (kb >= na) {
                cut = true;
                break;
            }
            int64_t qend = q0 + PROBE_TILE;
            if (qend > o + B) qend = o + B;
            ++tiles;
            int32_t head[4] = {0, 0, 0, 0};
            if (q0 > o) {  // prefix of both streams from the block origin up to the tile
                range_sums(F.data, n, o, q0, o, head[0], head[1]);
                range_sums(F.data, n, o + B, q0 + B, o, head[2], head[3]);
                block_reduce<4>(head, sh);
            }
            const int64_t p0 = q0 + (int64_t)t * PROBE_PPT;
            uint32_t xa[4], xb[4];
            load16(F.data, n, p0, xa);
            load16(F.data, n, p0 + B, xb);
            int32_t part[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < PROBE_PPT; ++i) {
                const int32_t va = sbyte_of(xa, i), vb = sbyte_of(xb, i);
                part[0] += va;
                part[1] += (int32_t)((uint32_t)(p0 + i - o) * (uint32_t)va);
                part[2] += vb;
                part[3] += (int32_t)((uint32_t)(p0 + B + i - o) * (uint32_t)vb);
            }
            int32_t pre[4] = {part[0], part[1], part[2], part[3]};
            block_exscan<4>(pre, sh);
            if (t == 0) s_hit = 0x7FFFFFFF;
            __syncthreads();
            uint32_t keys[PROBE_PPT];
            if (t < PROBE_THREADS && p0 < qend && p0 <= stop && p0 + PROBE_PPT > a) {
                const uint32_t pa = (uint32_t)(head[0] + pre[0]), pa2 = (uint32_t)(head[1] + pre[1]);
                const uint32_t pb = (uint32_t)(head[2] + pre[2]), pb2 = (uint32_t)(head[3] + pre[3]);
                const int32_t To = F.aw[kb];
                const uint32_t s1o = (uint32_t)To & 0xFFFFu, s2o = (uint32_t)To >> 16;
                const uint32_t P1e = s1o + pb;
                const uint32_t P2e = (uint32_t)B * s1o - s2o + pb2;  // windows inside [o, nB]: e0 = o + B
                const uint32_t s1 = P1e - pa;
                const uint32_t s2 = (uint32_t)(p0 + B - o) * s1 - (P2e - pa2);  // (p0 + B - o) s1 - sum (j - o) x_j
                int32_t R = (int32_t)((s1 & 0xFFFFu) | (s2 << 16));  // synced: the key is the true weak sum
#pragma unroll
                for (int i = 0; i < PROBE_PPT; ++i) {
                    keys[i] = (uint32_t)R;
                    R = roll_add(roll_sub(R, (int32_t)B, sbyte_of(xa, i)), sbyte_of(xb, i));
                }
                uint32_t valid = 0;
#pragma unroll
                for (int i = 0; i < PROBE_PPT; ++i) {
                    const int64_t pp = p0 + i;
                    if (pp >= a && pp <= stop && pp < qend) valid |= 1u << i;
                }
                const int h = chain_first_hit16(F.kslots, F.kmask, kset, keys, valid);
                if (h >= 0) atomicMin(&s_hit, (int32_t)(p0 + h - q0));
            }
            __syncthreads();
            if (s_hit != 0x7FFFFFFF && (s_hit >> 4) == t) {
#pragma unroll
                    for (int i = 0; i < PROBE_PPT; ++i)  // (a static index: keys stays in registers)
                        if (i == (s_hit & 15)) s_key = keys[i];
                }
            __syncthreads();
            if (s_hit != 0x7FFFFFFF) {
                p = q0 + s_hit;
                key = s_key;
            }
            __syncthreads();
            q0 = qend;
        }
        if (p < 0) {
            if (cut) {  // past the speculation: the rest of it (phase 1), or the host -- which also takes a
                // poisoned walk (phase 1 starts from the unpoisoned state)
                if (na < F.na && !poisoned) status = CHAIN_MORE;
                why = CHAIN_WHY_CUT;
                break;
            }
            if (f <= last) {  // a flush (quirk A): the host, which need not search [s, stop] again
                clear_to = stop;
                why = CHAIN_WHY_FLUSH;
                break;
            }
            emit_lit(m, n - m);           // no candidate before the end
            status = CHAIN_DONE;
            s = n;
            why = CHAIN_WHY_END;
            break;
        }
        // the event at p: its bucket (Multimap order), the candidates of Checksum.getCandidateChunks
        const int64_t te0 = chain_clock(timed);
        ++events;
        const int64_t kp = p / B;
        const bool spec_digest = !poisoned && p % B == 0 && kp < na;
        // An aligned hit on its own chunk (chain flag: the speculation's weak sum and digest are chunk kp's) whose weak
        // sum no other chunk has: the bucket is {kp}, closeIndexOf({kp}, pref) is kp, and the window's digest (the
        // speculation's) equals chunk kp's -- the match Checksum.getCandidateChunks + Sender.java:1257-1287 find, with
        // no round trip (config 4's 50%-modified form: every event of a walk on an unedited stretch)
        if (sc_hit && spec_digest && kp < C && s_sc[0] != 0 && !(kp == C - 1 && F.rem > 0)) {
            pf_s = p + B;
            pf_pref = (int32_t)(kp + 1);
            pf_flag = (uint8_t)s_sc[1];
            pf_aw = s_sc[2];
            pf_tw = s_sc[3];
            emit_lit(m, p - m);
            emit_match(p, B, (int32_t)kp, 1);
            pref = (int32_t)(kp + 1);
            s = m = p + B;
            poisoned = 0;
            t_event += chain_clock(timed) - te0;
            continue;
        }
        // the speculation's digest of an aligned window, loaded beside the bucket's slots (it depends only on p)
        // ... and chunk kp's own digest beside it: the candidate of a window that sits where its chunk sat (identical
        // stretches, edited blocks in place) is decided without another round trip
        uint32_t dgk[4] = {0u, 0u, 0u, 0u};
        const bool diag = spec_digest && kp < C;
        if (spec_digest) chain_digest_load(F.as + kp * dl, dl, dg);
        if (diag) chain_digest_load(F.table_strong + kp * dl, dl, dgk);
        if (spec_digest) {  // the next step's first words, should the window match its own chunk kp (s = p + B, pref = kp + 1)
            const int64_t kn = kp + 1;
            pf_s = p + B;
            pf_pref = (int32_t)kn;
            pf_flag = kn < nflags ? F.flags[kn] : (uint8_t)0;
            pf_aw = kn < na ? F.aw[kn] : 0;
            pf_tw = (kn < C && kn < na) ? F.table_weak[kn] : 0;
        }
        if (t < 64) {
            // every chunk with this key lies on the probe path before the first empty slot: wave 0 reads 64 slots of
            // it per round trip (one, nearly always) instead of one dependent load per slot
            int32_t cnt = 0;
            const unsigned long long* ks = F.kslots;
            uint32_t h = slot_hash(key) & F.kmask;
            for (bool more = true; more; h = (h + 64u) & F.kmask) {
                const unsigned long long v = ks[(h + (uint32_t)t) & F.kmask];
                const unsigned long long empty = __ballot(v == 0ull);
                const int lim = empty ? __builtin_ctzll(empty) : 64;  // slots before the first empty one
                const bool mine = t < lim && (uint32_t)(v >> 32) == key;
                const unsigned long long hits = __ballot(mine);
                const int at = cnt + __popcll(hits & ((1ull << t) - 1ull));
                if (mine && at < CHAIN_BUCKET_CAP) s_bk[at] = (int32_t)((uint32_t)v - 1u);
                cnt += __popcll(hits);
                more = empty == 0ull;
            }
            if (t == 0) {  // ascending chunk index (insertion order); the wave's LDS operations execute in order
                s_nbk = cnt;
                for (int i = 1; i < cnt && i < CHAIN_BUCKET_CAP; ++i)
                    for (int j = i; j > 0 && s_bk[j - 1] > s_bk[j]; --j) {
                        const int32_t x = s_bk[j];
                        s_bk[j] = s_bk[j - 1];
                        s_bk[j - 1] = x;
                    }
            }
        }
        __syncthreads();
        t_evb += chain_clock(timed) - te0;
        const int32_t size = s_nbk;
        if (size == 0 || size > CHAIN_BUCKET_CAP) {
            why = CHAIN_WHY_BUCKET;
            break;
        }
        // closeIndexOf(bucket, pref) (Checksum.java:175-213): pref's position, else the first index above it,
        // else the last; not length-filtered.  Then the others in ascending order with length == window.
        int32_t l = 0, r = size - 1, init = -1;
        while (l <= r) {
            const int32_t mid = l + (r - l) / 2;
            if (s_bk[mid] == pref) {
                init = mid;
                break;
            }
            if (s_bk[mid] < pref) l = mid + 1;
            else r = mid - 1;
        }
        if (init < 0) init = l < size - 1 ? l : size - 1;
        const int64_t w = B;  // p <= nB
        // Sender.java:1259-1263: the window's digest -- the speculation's at aligned positions, else one lane digests
        // the window here (lane_chunk_sums over the B bytes at p, the seed appended), the host path's md5_at
        const uint8_t* md5c = poisoned ? stale : F.as + kp * dl;
        if (!spec_digest && !poisoned) {
            const int64_t td0 = chain_clock(timed);
            chain_window_digest(F.data + p, (uint32_t)B, (uint32_t)dl, F.seed, s_win, s_dig);  // (ends with a barrier)
            md5c = s_dig;
            chain_digest_load(s_dig, dl, dg);
            ++digests;
            t_digest += chain_clock(timed) - td0;
        }
        int32_t hit = -1;
        for (int32_t it = -1; it < size && hit < 0; ++it) {
            int32_t pos;
            if (it < 0) {
                pos = init;
            } else {
                const int32_t c = s_bk[it];
                const int64_t clen = (c == C - 1 && F.rem > 0) ? F.rem : B;  // Checksum.java:197-203
                if (it == init || clen != w) continue;
                pos = it;
            }
            const int32_t c = s_bk[pos];
            const bool eq = (diag && c == kp) ? ((dg[0] ^ dgk[0]) | (dg[1] ^ dgk[1]) | (dg[2] ^ dgk[2]) | (dg[3] ^ dgk[3])) == 0u
                                              : chain_digest_eq_reg(dg, F.table_strong + (int64_t)c * dl, dl);
            if (eq) hit = c;
        }
        __syncthreads();
        t_event += chain_clock(timed) - te0;
        if (hit < 0) {
            // the cached digest is stale from here on (quirk B): the walk goes on with it from p + 1, comparing every
            // later candidate with it, up to the next flush point (a hit at the flush point itself flushes there: the
            // host retakes that step from s)
            if (p < f) {
                s = p + 1;
                if (poisoned) continue;  // (already stale: nothing changes)
                poisoned = 1;
                stale = md5c;
                // no chunk carries the stale digest: nothing can match again (the host's closed form), so the
                // file needs no more speculation
                if (t == 0) s_any = 0;
                __syncthreads();
                {  // the stale digest is in dg; two chunks' digests per thread in flight at a time
                    bool any = false;
                    for (int64_t c = t; c < C; c += 2 * CHAIN_THREADS) {
                        const int64_t c2 = c + CHAIN_THREADS < C ? c + CHAIN_THREADS : c;
                        any |= (int)chain_digest_eq_reg(dg, F.table_strong + c * dl, dl) |
                               (int)chain_digest_eq_reg(dg, F.table_strong + c2 * dl, dl);
                    }
                    if (any) s_any = 1;
                }
                __syncthreads();
                dead = s_any == 0;
                // dead: the host's closed form (resolver.cpp), here when its literals fit the event buffer -- the
                // flushes at mark + 9B (one 10B literal each), then the rest (Sender.java:1313-1316)
                if (dead) {
                    const int64_t nfl = s <= last ? (n - m) / (10 * B) : 0;  // (the loop has ended: no flushes)
                    if (nev + nfl + 3 <= F.ev_cap) {
                        flush_pend();  // the literals themselves: one per thread (writes to pinned host memory)
                        drain_ev();
                        for (int64_t i = t; i < nfl; i += CHAIN_THREADS)
                            F.ev[nev + i] = rsh_event{m + 10 * B * i, 10 * B, RSH_EV_LITERAL, 0, 0, 0};
                        nev += (int32_t)nfl;
                        nev_w = nev;
                        lit += 10 * B * nfl;
                        m += 10 * B * nfl;
                        flushes += nfl;
                        emit_lit(m, n - m);
                        s = n;
                        status = CHAIN_DONE;
                        poisoned = 0;
                    }
                }
                if (!dead) continue;  // some chunk carries it: the search goes on from p + 1
                why = status == CHAIN_DONE ? CHAIN_WHY_CLOSED : CHAIN_WHY_DEADCAP;
            } else {
                // the candidate sits on the flush point itself: Java takes the flush there (FileView.isFull,
                // Sender.java:1294-1310) with the window's digest cached (quirk B).  The walk takes it too -- the
                // literal up to f + B, then the rolling value slid by a whole window (quirk A) -- and hands the
                // desynced state over (E at s2 = f + B): the resolver probes the rest of the file with the stale
                // digest's keys and the batched flush chain in one round trip
                if (!poisoned) {
                    poisoned = 1;
                    stale = md5c;
                }
                emit_lit(m, p + B - m);
                ++flushes;
                const int64_t s2 = p + B;
                s = m = s2;
                if (s2 <= last) {
                    const int32_t jx = (int32_t)(int8_t)F.data[p];
                    uint32_t rlo = (key & 0xFFFFu) - (uint32_t)jx, rhi = (key >> 16) - (uint32_t)B * (uint32_t)jx;
                    if (n - s2 >= B) {  // :1308-1310: the window at s2 is full -- its new last byte goes in
                        rlo += (uint32_t)(int32_t)(int8_t)F.data[s2 + B - 1];
                        rhi += rlo;
                    }
                    uint32_t T2;
                    if (s2 % B == 0 && s2 / B < na) {
                        T2 = (uint32_t)F.aw[s2 / B];
                    } else {  // T(s2) over its window, min(B, n - s2) bytes
                        const int64_t L2 = n - s2 < B ? n - s2 : B;
                        int32_t w2[2] = {0, 0};
                        range_sums(F.data, n, s2, s2 + L2, s2, w2[0], w2[1]);
                        block_reduce<2>(w2, sh);
                        const uint32_t S1 = (uint32_t)w2[0], S2 = (uint32_t)L2 * S1 - (uint32_t)w2[1];
                        T2 = (S1 & 0xFFFFu) | (S2 << 16);
                    }
                    desync_lo = (rlo - T2) & 0xFFFFu;
                    desync_hi = (rhi - (T2 >> 16)) & 0xFFFFu;
                }
                why = CHAIN_WHY_FLUSHED;
            }
            break;
        }
        emit_lit(m, p - m);  // Sender.java:1265-1288
        emit_match(p, w, hit, 1);
        pref = hit + 1;
        s = m = p + w;
        poisoned = 0;  // a match clears the cached digest (Sender.java:1287)
    }
    flush_pend();
    drain_ev();
    if (t == 0) {
        out->s = s;
        out->m = m;
        out->pref = pref;
        out->status = status;
        out->n_ev = nev;
        out->tiles = tiles;
        out->digests = digests;
        out->flushes = flushes;
        out->t_total += chain_clock(timed) - tk0;
        out->t_tiles += t_tiles;
        out->t_check += t_check;
        out->t_event += t_event;
        out->t_digest += t_digest;
        out->t_kset += t_kset;
        out->t_chain += t_chain;
        out->t_drain += t_drain;
        out->t_evb += t_evb;
        out->spec_full = phase == 1;
        out->mapped = mapped;
        out->clear_to = clear_to;
        out->why = why;
        out->elo = desync_lo;
        out->ehi = desync_hi;
        out->first_mapped = first_mapped;
        // a file that needs no more speculation stops its phase-1 K1 groups (they poll this word); any other stop
        // keeps them (the resolver's aligned lookups past the prefix use them)
        const bool stop_spec = phase == 0 && F.abort && (status == CHAIN_DONE || dead);
        out->aborted = stop_spec;
        if (stop_spec) *(volatile int*)F.abort = abort_gen;
        out->md5c_valid = poisoned;
        if (poisoned)
            for (int j = 0; j < dl && j < 16; ++j) out->md5c[j] = stale[j];
        out->literal = lit;
        out->matched = mat;
        out->chain_matches = chain_matches;
        out->events = events;
        __threadfence_system();  // the record and the events (drained above) before the completion word
        *(volatile int32_t*)&out->fin = 1;
    }
    if (H != nullptr) {  // this walk is over: its helpers stop, and the workgroup helps the walks still searching
        if (t == 0) chain_st(&H->live, 0);
        __syncthreads();
        chain_help(files, nfiles, (uint32_t)abort_gen, help, s_ck, &s_ck_full, sh, s_seg, &s_best, &s_word, &s_live,
                   timed != 0);
    }
}

hipError_t launch_chain_advance(const ChainFile* files, uint32_t nfiles, hipStream_t s, int phase, int abort_gen,
                                ChainHelp* help, uint32_t helpers, bool timed) {
    if (nfiles == 0) return hipSuccess;
    if (phase != 0 || help == nullptr || nfiles >= (1u << 20)) {  // (helpers pick files by a 20-bit index)
        help = nullptr;
        helpers = 0;
    }
    hipLaunchKernelGGL(chain_advance_kernel, dim3(nfiles + helpers), dim3(CHAIN_THREADS), 0, s, files, phase,
                       abort_gen, help, (int)nfiles, timed ? 1 : 0);
    return hipGetLastError();
}

// The chunk index of the chain walk: every chunk i of a file as (key << 32) | (i + 1) in an open-addressing table
// (0 = empty); the chunks with one key all lie on that key's probe path before its first empty slot.
// A thread's keys go in groups of CHUNK_INDEX_MLP: the group's first-slot CASes are issued back to back (independent
// atomics, all in flight at once), and only a CAS that found its slot taken walks the probe path (a serial
// CAS-then-next loop keeps one atomic round trip in flight per thread).  Config 4's 2 M chunks on the background
// grid beside the prefix K1: the index now ends inside that launch instead of 0.03 ms after it.
// Duplicates: of two chunks with one key, the one that ends further along the path found the other's slot taken (its
// CAS there returned the other's entry), so a failed CAS that returns the inserting chunk's own key marks both chunks;
// every chunk whose key another chunk has is marked so, at no cost beyond the CASes the insert takes anyway.
constexpr int CHUNK_INDEX_MLP = 8;
__global__ void chunk_index_kernel(const ChunkIndexEnt* __restrict__ ents, uint32_t nfiles) {
    const TableEnt e = ents[blockIdx.y].t;
    uint8_t* const dup = ents[blockIdx.y].dup;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < e.nkeys; i0 += CHUNK_INDEX_MLP * stride) {
        unsigned long long v[CHUNK_INDEX_MLP], got[CHUNK_INDEX_MLP];
        uint32_t h[CHUNK_INDEX_MLP];
#pragma unroll
        for (int j = 0; j < CHUNK_INDEX_MLP; ++j) {
            const int64_t i = i0 + j * stride;
            const uint32_t key = i < e.nkeys ? (uint32_t)e.keys[i] : 0u;
            v[j] = ((unsigned long long)key << 32) | (uint32_t)(i + 1);
            h[j] = slot_hash(key) & e.mask;
        }
#pragma unroll
        for (int j = 0; j < CHUNK_INDEX_MLP; ++j)
            got[j] = i0 + j * stride < e.nkeys ? atomicCAS(&e.slots[h[j]], 0ull, v[j]) : 0ull;
#pragma unroll
        for (int j = 0; j < CHUNK_INDEX_MLP; ++j) {
            unsigned long long g = got[j];
            uint32_t hh = h[j];
            while (g != 0ull) {
                if ((g >> 32) == (v[j] >> 32)) {  // another chunk with this key: both are duplicates
                    dup[(uint32_t)v[j] - 1] = 1;
                    dup[(uint32_t)g - 1] = 1;
                }
                hh = (hh + 1) & e.mask;
                g = atomicCAS(&e.slots[hh], 0ull, v[j]);
            }
        }
    }
    (void)nfiles;
}

hipError_t launch_chunk_index(const ChunkIndexEnt* ents, uint32_t nfiles, int32_t max_keys, hipStream_t s, bool bg) {
    if (nfiles == 0 || max_keys <= 0) return hipSuccess;
    const uint32_t gx = (uint32_t)std::min<int64_t>((max_keys + 255) / 256, bg ? 2 : 64);
    hipLaunchKernelGGL(chunk_index_kernel, dim3(gx, nfiles), dim3(256), 0, s, ents, nfiles);
    return hipGetLastError();
}
// A kernel that does nothing: its first launch makes the runtime load this file's code object (the chain walk) on a
// fresh context, which rsh_ctx_create pays instead of the first segment scan (launch_warm).
__global__ void warm_chain_kernel() {}
// Scratch: chain_advance_kernel spills ~572 B per lane (256 VGPRs at two waves per SIMD) and its out-of-line helpers
// keep their saved registers there.  The runtime sizes a queue's scratch at the first dispatch that needs it, which held
// up the first segment scan's walk by ~0.7 ms; this kernel needs more per lane than the walk, over as many waves as a
// walk launch can have (256 workgroups of 512), so rsh_ctx_create pays that instead (on the context stream, the walk's).
constexpr int kWarmScratchWords = 160;  // 640 B per lane
__global__ __launch_bounds__(CHAIN_THREADS) void warm_scratch_kernel(int32_t sel, int32_t* out) {
    volatile int32_t a[kWarmScratchWords];
    for (int i = 0; i < kWarmScratchWords; ++i) a[i] = i ^ sel;
    const int32_t v = a[(threadIdx.x + (uint32_t)sel) % kWarmScratchWords];
    if (out && v == 0x7FFFFFFF) out[0] = v;  // never taken (out is null): keeps the array
}
hipError_t launch_warm_chain(hipStream_t s) {
    hipLaunchKernelGGL(warm_chain_kernel, dim3(1), dim3(64), 0, s);
    hipLaunchKernelGGL(warm_scratch_kernel, dim3(256), dim3(CHAIN_THREADS), 0, s, 1, nullptr);
    return hipGetLastError();
}

}  // namespace rsh
