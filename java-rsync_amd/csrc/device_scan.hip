// device_scan.hip -- gfx950 kernels of the Sender's search: the probe hash table, the range probes (first hit of a
// rolling key in an interval, hit windows and buckets), the pass-free long probe and the batched flush chain.  The
// batched scan's chain walk is in device_chain.hip, the K1 kernels in device.hip, the copies and gathers in
// device_io.hip.  See DESIGN.md sections 4-5.
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
// Probe table (distinct weak keys).  Slot = (1 << 32) | key; 0 = empty.
// ------------------------------------------------------------------------------------------------

__global__ void table_clear_kernel(unsigned long long* slots, uint64_t nslots, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(3);
    for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x) slots[i] = 0ull;
}

__global__ void table_insert_kernel(unsigned long long* slots, uint32_t mask, const int32_t* __restrict__ keys,
                                    uint32_t nkeys) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys) return;
    const uint32_t key = (uint32_t)keys[i];
    const unsigned long long v = (1ull << 32) | key;
    uint32_t h = slot_hash(key) & mask;
    for (uint32_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long prev = atomicCAS(&slots[h], 0ull, v);
        if (prev == 0ull || prev == v) return;
        h = (h + 1) & mask;
    }
}

hipError_t launch_table_clear(unsigned long long* d_slots, uint64_t nslots, hipStream_t s, bool bg) {
    const uint64_t cap = bg ? kBackgroundGroups : 2048u;
    hipLaunchKernelGGL(table_clear_kernel, dim3((uint32_t)std::min<uint64_t>((nslots + 255) / 256, cap)), dim3(256), 0, s,
                       d_slots, nslots, bg ? 0 : 1);
    return hipGetLastError();
}

hipError_t launch_table_insert(unsigned long long* d_slots, uint32_t mask, const int32_t* d_keys, uint32_t nkeys,
                               hipStream_t s) {
    if (nkeys == 0) return hipSuccess;
    hipLaunchKernelGGL(table_insert_kernel, dim3((nkeys + 255) / 256), dim3(256), 0, s, d_slots, mask, d_keys,
                       nkeys);
    return hipGetLastError();
}

__device__ __forceinline__ bool table_has(const ProbeTable& t, uint32_t key) {
    const unsigned long long v = (1ull << 32) | key;
    uint32_t h = slot_hash(key) & t.mask;
    for (;;) {
        const unsigned long long sl = t.slots[h];
        if (sl == v) return true;
        if (sl == 0ull) return false;
        h = (h + 1) & t.mask;
    }
}

// ------------------------------------------------------------------------------------------------
// Probe: first position in [a, b) whose Sender rolling key hits the table.  Positions are tiled in
// aligned-block coordinates (block k = [kB, kB + B), tile = 4096 positions); one 256-lane workgroup per
// tile, 16 positions per lane.  With o = kB and P1/P2 the prefix sums of x and (j - o) x from o:
//   T(p) = (s1, s2),  s1 = P1(e) - P1(p),  s2 = (e - o) s1 - (P2(e) - P2(p)),  e = min(p + B, n),
// and P1(o + B) = s1(o), P2(o + B) = B s1(o) - s2(o) from the source's own aligned sum T(o).  Lane start
// values come from the workgroup's prefix of both streams (x[p] and x[p + B]); each lane then rolls its
// 16 positions with the exact Java updates (Rolling.java:25-60) on R = T + E.
// ------------------------------------------------------------------------------------------------

// A lane's 16 keys at positions base + i (bit i of valid: in the interval): every hit goes to the file's hit list
// (the first position by atomicMin, up to PROBE_HITS_CAP of them listed).  The stale digest's few keys (the batched
// flush chain's probes over a file's rest) are compared against each key in turn; otherwise the 16 first hash slots
// go out in one burst of independent loads -- most keys are decided by their first slot (load factor <= 1/2), so a
// lane waits for about one L2 round trip -- and only keys whose first slot holds another key walk the probe path.
// Branch free but for those walks and the (rare) hits.
__device__ __forceinline__ void probe_check16(const ScanFile& F, const ProbeTable& table, int nsmall,
                                              const uint32_t (&key)[16], uint32_t valid, int64_t base) {
    uint32_t m = 0;
    if (nsmall > 0) {
        // one compare per key and position into a lane mask (the scalar unit ORs them); which positions only when
        // some lane matched (rare: a stale digest's keys over a file's rest)
        bool any = false;
        for (int j = 0; j < nsmall; ++j) {
            const uint32_t kj = F.small[j];
#pragma unroll
            for (int i = 0; i < 16; ++i) any |= key[i] == kj;
        }
        if (__builtin_expect(any, 0))
            for (int j = 0; j < nsmall; ++j) {
                const uint32_t kj = F.small[j];
#pragma unroll
                for (int i = 0; i < 16; ++i) m |= (uint32_t)(key[i] == kj) << i;
            }
    } else {
        unsigned long long sl[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) sl[i] = (valid >> i) & 1u ? table.slots[slot_hash(key[i]) & table.mask] : 0ull;
        uint32_t need = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (sl[i] == ((1ull << 32) | key[i])) m |= 1u << i;
            else if (sl[i] != 0ull) need |= 1u << i;
        }
        need &= valid;
        while (need) {
            const int i = __builtin_ctz(need);
            uint32_t kk = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (j == i) kk = key[j];
            if (table_has(table, kk)) m |= 1u << i;
            need &= need - 1u;
        }
    }
    m &= valid;
    while (m) {
        const int i = __builtin_ctz(m);
        uint32_t kk = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j == i) kk = key[j];
        const int64_t p = base + i;
        atomicMin(&F.out->first, (unsigned long long)p);
        const unsigned long long at = atomicAdd(&F.out->count, 1ull);
        if (at < (unsigned long long)PROBE_HITS_CAP) {
            F.out->pos[at] = (unsigned long long)p;
            F.out->key[at] = kk;
        }
        m &= m - 1u;
    }
}

// bit i set for positions base + i in [lo, hi), i < 16
__device__ __forceinline__ uint32_t probe_valid16(int64_t base, int64_t lo, int64_t hi) {
    const int64_t a = lo - base, b = hi - base;
    if (b <= 0 || a >= 16 || b <= a) return 0u;
    const int ia = a < 0 ? 0 : (int)a, ib = b > 16 ? 16 : (int)b;
    return (0xFFFFu >> (16 - ib)) & (0xFFFFu << ia);
}

__global__ __launch_bounds__(PROBE_THREADS) void probe_first_kernel(ProbeArgs A) {
    __builtin_amdgcn_s_setprio(3);  // resolver latency path: ahead of a co-running speculation launch
    __shared__ int32_t sh[4 * PROBE_THREADS / 64];
    const ProbeTile tile = A.tiles[blockIdx.x];
    const ProbeIv I = A.ivs[tile.iv];
    const ScanFile& F = A.files[I.file];
    const int64_t n = F.n, B = F.B;
    const uint8_t* __restrict__ data = F.data;
    const ProbeTable table{F.slots, F.mask};
    const int64_t k = tile.q0 / B;
    const int64_t o = k * B;
    const int64_t q0 = tile.q0;
    int64_t qend = q0 + PROBE_TILE;
    if (qend > o + B) qend = o + B;
    if (q0 >= I.b || qend <= I.a || q0 >= n) return;  // uniform over the workgroup

    // prefix of both streams from the block origin up to the tile: the partial sums of the tiles before it
    int32_t head[4] = {0, 0, 0, 0};
    const int ti = (int)((q0 - o) / PROBE_TILE);
    if (ti > 0) {
        if (tile.pbase < 0) {  // near the block start: re-read the <= PROBE_INLINE_TILES tiles before it
            range_sums(data, n, o, q0, o, head[0], head[1]);
            range_sums(data, n, o + B, q0 + B, o, head[2], head[3]);
        } else if (threadIdx.x < ti) {
            const int4 v = A.partials[tile.pbase + threadIdx.x];
            head[0] = v.x;
            head[1] = v.y;
            head[2] = v.z;
            head[3] = v.w;
        }
        block_reduce<4>(head, sh);
    }

    const int t = threadIdx.x;
    const int64_t p0 = q0 + (int64_t)t * PROBE_PPT;
    uint32_t xa[4], xb[4];
    load16(data, n, p0, xa);
    load16(data, n, p0 + B, xb);
    int32_t part[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int32_t va = (p0 + i < n) ? sbyte_of(xa, i) : 0;
        const int32_t vb = (p0 + B + i < n) ? sbyte_of(xb, i) : 0;
        part[0] += va;
        part[1] += (int32_t)((uint32_t)(p0 + i - o) * (uint32_t)va);
        part[2] += vb;
        part[3] += (int32_t)((uint32_t)(p0 + B + i - o) * (uint32_t)vb);
    }
    int32_t pre[4] = {part[0], part[1], part[2], part[3]};
    block_exscan<4>(pre, sh);
    if (p0 >= qend || p0 >= I.b || p0 + PROBE_PPT <= I.a) return;

    const uint32_t pa = (uint32_t)(head[0] + pre[0]), pa2 = (uint32_t)(head[1] + pre[1]);  // P1(p0), P2(p0)
    const uint32_t pb = (uint32_t)(head[2] + pre[2]), pb2 = (uint32_t)(head[3] + pre[3]);  // sums over [o+B, p0+B)
    const int32_t To = F.aligned_weak[k];
    const int64_t e0 = (o + B < n ? o + B : n);
    const uint32_t s1o = (uint32_t)To & 0xFFFFu, s2o = (uint32_t)To >> 16;
    const uint32_t P1e = s1o + pb;
    const uint32_t P2e = (uint32_t)(e0 - o) * s1o - s2o + pb2;
    const int64_t endq = (p0 + B < n ? p0 + B : n);
    const uint32_t s1 = P1e - pa;
    const uint32_t s2 = (uint32_t)(endq - o) * s1 - (P2e - pa2);
    const int64_t nb = n - B;
    auto clampB = [&](int64_t p) { return p < nb ? p : nb; };
    const uint32_t ehi = I.e_hi + I.e_lo * (uint32_t)(clampB(p0) - clampB(I.anchor));
    int32_t R = (int32_t)(((s1 + I.e_lo) & 0xFFFFu) | ((s2 + ehi) << 16));
    // keys of all 16 positions first (ALU only), then their first hash slots in one burst of independent
    // loads: a hit/miss is decided by the first slot for most keys (load factor <= 1/2), so a lane waits
    // for about one L2 round trip instead of 16 serial ones
    uint32_t key[PROBE_PPT];
#pragma unroll
    for (int i = 0; i < PROBE_PPT; ++i) {
        key[i] = (uint32_t)R;
        const int64_t p = p0 + i;
        const int64_t w = (n - p < B ? n - p : B);
        R = roll_sub(R, (int32_t)w, sbyte_of(xa, i));
        if (n - (p + 1) >= B) R = roll_add(R, sbyte_of(xb, i));
    }
    probe_check16(F, table, F.nsmall, key, probe_valid16(p0, I.a, I.b < qend ? I.b : qend), p0);
}

__global__ void probe_out_reset_kernel(ProbeOut* out, uint32_t n) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        out[i].first = ~0ull;
        out[i].count = 0ull;
    }
}

hipError_t launch_probe_out_reset(ProbeOut* d_out, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(probe_out_reset_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d_out, n);
    return hipGetLastError();
}

// Pass 1: one workgroup per partial tile [q0, min(q0 + PROBE_TILE, o + B)), o = its block start.
__global__ __launch_bounds__(256) void probe_partials_kernel(const ScanFile* __restrict__ files,
                                                             const PartialTile* __restrict__ pt,
                                                             int4* __restrict__ out) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[4 * 256 / 64];
    const PartialTile t = pt[blockIdx.x];
    const ScanFile& F = files[t.file];
    const int64_t B = F.B, q0 = t.q0;
    const int64_t o = q0 / B * B;
    const int64_t qe = q0 + PROBE_TILE < o + B ? q0 + PROBE_TILE : o + B;
    int32_t v[4] = {0, 0, 0, 0};
    range_sums(F.data, F.n, q0, qe, o, v[0], v[1]);
    range_sums(F.data, F.n, q0 + B, qe + B, o, v[2], v[3]);
    block_reduce<4>(v, sh);
    if (threadIdx.x == 0) out[blockIdx.x] = make_int4(v[0], v[1], v[2], v[3]);
}

void probe_partials(std::vector<ProbeTile>* tiles, size_t t0, int64_t B, int32_t file, std::vector<PartialTile>* out) {
    int64_t cur_block = -1, covered = 0;  // tiles of cur_block already listed: [0, covered)
    int32_t base = 0;
    for (size_t i = t0; i < tiles->size(); ++i) {
        ProbeTile& t = (*tiles)[i];
        const int64_t k = t.q0 / B;
        const int64_t ti = (t.q0 - k * B) / PROBE_TILE;
        if (k != cur_block) {  // one file's tiles arrive in increasing position order
            cur_block = k;
            covered = 0;
            base = (int32_t)out->size();
        }
        if (ti <= PROBE_INLINE_TILES) {  // the kernel re-reads the few tiles before it (no pass 1)
            t.pbase = -1;
            continue;
        }
        for (; covered < ti; ++covered) out->push_back(PartialTile{k * B + covered * PROBE_TILE, file, 0});
        t.pbase = base;
    }
}

// grid (1 + 16 W + NEXT_SUMS_MAX, nreq): block 0 computes T(p) and the key, blocks 1..16 W copy the windows,
// the last ones T(p + k B) for k <= next_sums (the phase guess's checks, in parallel with T(p)).
__global__ __launch_bounds__(256) void hit_window_kernel(const ScanFile* __restrict__ files,
                                                         const ProbeIv* __restrict__ ivs,
                                                         const int32_t* __restrict__ req) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[2 * 256 / 64];
    const ScanFile& F = files[req[blockIdx.y]];
    const unsigned long long f = F.out->first;
    if (f == ~0ull) return;
    const int64_t n = F.n, B = F.B;
    const uint8_t* __restrict__ data = F.data;
    const int64_t p = (int64_t)f;
    const int64_t w = (n - p < B ? n - p : B);
    if (blockIdx.x == 0) {
        int32_t v[2] = {0, 0};
        range_sums(data, n, p, p + w, p, v[0], v[1]);
        block_reduce<2>(v, sh);
        if (threadIdx.x == 0) {
            const uint32_t S1 = (uint32_t)v[0];
            const uint32_t S2 = (uint32_t)w * S1 - (uint32_t)v[1];
            const int32_t T = (int32_t)((S1 & 0xFFFFu) | (S2 << 16));
            *reinterpret_cast<int32_t*>(F.hit) = T;
            // the file's interval holding p (disjoint, ascending) gives E(p); R = T + E is the key that hit
            int32_t lo = F.iv0, hi = F.iv0 + F.niv - 1;
            while (lo < hi) {
                const int32_t mid = (lo + hi + 1) / 2;
                if (ivs[mid].a <= p) lo = mid;
                else hi = mid - 1;
            }
            const ProbeIv I = ivs[lo];
            const int64_t nb = n - B;
            const int64_t cp = p < nb ? p : nb, ca = I.anchor < nb ? I.anchor : nb;
            const uint32_t ehi = I.e_hi + I.e_lo * (uint32_t)(cp - ca);
            F.bucket[0] = 0;
            F.bucket[1] = (int32_t)((((uint32_t)T + I.e_lo) & 0xFFFFu) | ((((uint32_t)T >> 16) + ehi) << 16));
        }
        if (threadIdx.x < PROBE_HITS_CAP) F.bucket[2 + HIT_BUCKET_CAP + (1 + LISTED_IDX) * threadIdx.x] = 0;
        return;
    }
    if (blockIdx.x > 16 * HIT_WINDOWS) {  // block 16 W + k: the window at p + k B (the next_sums that follow it)
        const int k = (int)(blockIdx.x - 16 * HIT_WINDOWS);
        if (k > F.next_sums) return;
        const int64_t pk = p + k * B, wk = n - pk < B ? n - pk : B;
        int32_t u[2] = {0, 0};
        if (wk > 0) range_sums(data, n, pk, pk + wk, pk, u[0], u[1]);
        block_reduce<2>(u, sh);
        if (threadIdx.x == 0) {
            const uint32_t S1 = (uint32_t)u[0];
            const uint32_t S2 = (uint32_t)(wk > 0 ? wk : 0) * S1 - (uint32_t)u[1];
            reinterpret_cast<int32_t*>(F.hit)[k] = (int32_t)((S1 & 0xFFFFu) | (S2 << 16));
        }
        return;
    }
    // blocks 1 + 16 k .. 16 k + 16 copy window k: the k-th smallest listed hit (k = 0 is the first hit; the
    // others only when the list is complete), so the resolver has the digest input of the next few
    // events the hit list answers without another round trip
    const int slot = (int)(blockIdx.x - 1) / 16, part = (int)(blockIdx.x - 1) % 16;
    if (slot >= F.nwin) return;
    int64_t pw = p;
    if (slot > 0) {
        const unsigned long long cnt = F.out->count;
        if (cnt > (unsigned long long)PROBE_HITS_CAP || (unsigned long long)slot >= cnt) return;
        __shared__ long long sel;
        if (threadIdx.x == 0) sel = -1;
        __syncthreads();
        if (threadIdx.x < (int)cnt) {  // rank of entry t among the listed positions (distinct)
            const unsigned long long me = F.out->pos[threadIdx.x];
            int rank = 0;
            for (int j = 0; j < (int)cnt; ++j) rank += F.out->pos[j] < me;
            if (rank == slot) sel = (long long)me;
        }
        __syncthreads();
        pw = (int64_t)sel;
        if (pw < 0) return;
    }
    const int64_t ww = (n - pw < B ? n - pw : B);
    uint8_t* __restrict__ h_win = F.hit + 16 + (int64_t)slot * B;
    for (int64_t o = 16 * ((int64_t)part * blockDim.x + threadIdx.x); o < ww; o += 16 * 16 * (int64_t)blockDim.x) {
        if (o + 16 <= ww) {
            uint32_t q[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 16; ++i) q[i >> 2] |= (uint32_t)data[pw + o + i] << (8 * (i & 3));
            *reinterpret_cast<uint4*>(h_win + o) = make_uint4(q[0], q[1], q[2], q[3]);
        } else {
            for (int64_t i = o; i < ww; ++i) h_win[i] = data[pw + i];
        }
    }
}

// The bucket of the hit key: chunk indices i with weak[i] == key (8 per lane); grid (., nreq).
__global__ __launch_bounds__(256) void hit_bucket_kernel(const ScanFile* __restrict__ files,
                                                         const int32_t* __restrict__ req) {
    __builtin_amdgcn_s_setprio(3);
    const ScanFile& F = files[req[blockIdx.y]];
    if (F.out->first == ~0ull) return;
    const int32_t C = F.C;
    const int32_t i0 = 8 * (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    const int32_t key = F.bucket[1];
    const int32_t* __restrict__ weak = F.table_weak;
    // the listed hits' keys too (complete lists only): their buckets spare the host a lookup per event
    // the hit list answers
    __shared__ int32_t lkey[PROBE_HITS_CAP];
    const unsigned long long cnt = F.out->count;
    const int nl = cnt <= (unsigned long long)PROBE_HITS_CAP ? (int)cnt : 0;
    if (threadIdx.x < nl) lkey[threadIdx.x] = (int32_t)F.out->key[threadIdx.x];
    __syncthreads();
    int32_t* __restrict__ lb = F.bucket + 2 + HIT_BUCKET_CAP;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int32_t i = i0 + k;
        if (i >= C) break;
        const int32_t wk = weak[i];
        if (wk == key) {
            const int32_t at = atomicAdd(&F.bucket[0], 1);
            if (at < HIT_BUCKET_CAP) F.bucket[2 + at] = i;
        }
        for (int j = 0; j < nl; ++j)
            if (wk == lkey[j]) {
                const int32_t at = atomicAdd(&lb[(1 + LISTED_IDX) * j], 1);
                if (at < LISTED_IDX) lb[(1 + LISTED_IDX) * j + 1 + at] = i;
            }
    }
}

hipError_t launch_hit_window(const ScanFile* files, const ProbeIv* ivs, const int32_t* req, int32_t nreq, int32_t max_C,
                             hipStream_t s) {
    if (nreq <= 0) return hipSuccess;
    hipLaunchKernelGGL(hit_window_kernel, dim3(1 + 16 * HIT_WINDOWS + NEXT_SUMS_MAX, (uint32_t)nreq), dim3(256), 0, s, files, ivs, req);
    if (max_C > 0)
        hipLaunchKernelGGL(hit_bucket_kernel, dim3((uint32_t)((max_C + 8 * 256 - 1) / (8 * 256)), (uint32_t)nreq),
                           dim3(256), 0, s, files, req);
    return hipGetLastError();
}

void probe_tiles(int64_t a, int64_t b, int64_t B, int32_t iv, std::vector<ProbeTile>* out) {
    if (a >= b) return;
    for (int64_t k = a / B; k <= (b - 1) / B; ++k) {
        const int64_t o = k * B;
        const int64_t lo = a > o ? a : o;
        const int64_t hi = b < o + B ? b : o + B;
        for (int64_t t = (lo - o) / PROBE_TILE; t <= (hi - 1 - o) / PROBE_TILE; ++t)
            out->push_back(ProbeTile{o + t * PROBE_TILE, iv, -1});
    }
}

int64_t probe_seg_len(int64_t full_positions, int64_t B) {
    // segments pay off for big probes (a flush chain over a file's rest) at block lengths whose anchor (B bytes per
    // workgroup) is small against the segment; a few long intervals keep the tiles' parallelism instead (a probe
    // beside the speculation K1 sits on the resolver's latency path: 128 KiB blocks as 8-pass segments were 1 ms
    // slower per config-5 step than as tiles)
    if (opt(OPT_PROBE_LONG) == 0 || B > PROBE_LONG_MAX_B || full_positions < PROBE_LONG_BIG) return 0;
    // ~1024 workgroups per unit of the option (one residency wave at 4 waves per SIMD), then longer ones
    const int64_t passes = full_positions / (1024 * opt(OPT_PROBE_LONG) * PROBE_LONG_SUB);
    return (passes < 1 ? 1 : passes > PROBE_LONG_PASSES ? PROBE_LONG_PASSES : passes) * PROBE_LONG_SUB;
}

int64_t probe_full_positions(int64_t a, int64_t b, int64_t n, int64_t B) {
    const int64_t e = b < n - B + 1 ? b : n - B + 1;
    return e > a ? e - a : 0;
}

void probe_plan(int64_t a, int64_t b, int64_t n, int64_t B, int32_t iv, int64_t seg_len, std::vector<ProbeTile>* tiles,
                std::vector<ProbeSeg>* segs) {
    const int64_t full_end = b < n - B + 1 ? b : n - B + 1;  // positions below it have a full window
    if (seg_len <= 0 || full_end - a < PROBE_LONG_MIN) {
        probe_tiles(a, b, B, iv, tiles);
        return;
    }
    for (int64_t q = a & ~(int64_t)15; q < full_end; q += seg_len)
        segs->push_back(ProbeSeg{q, iv, (int32_t)(full_end - q < seg_len ? full_end - q : seg_len)});
    probe_tiles(full_end, b, B, iv, tiles);  // the shrinking windows near the end, if the interval reaches them
}

// Pass-free probe over long segments (see ProbeSeg): T(q0) digested by the workgroup once, then sub-segments of
// PROBE_LONG_SUB positions in order: the lanes' start values from one exscan of their 64 positions' byte sums (both
// streams, weights relative to the sub-segment's start), each lane rolls its 64 positions with the exact Java updates
// on R = T + E and checks every key as probe_first_kernel does per tile, and the last lane's rolled value (less E)
// anchors the next sub-segment.  One anchor and one launch slot per segment (up to PROBE_LONG_PASSES passes).
__global__ __launch_bounds__(PROBE_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void probe_long_kernel(ProbeArgs A, const ProbeSeg* __restrict__ segs) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[4 * PROBE_THREADS / 64];
    __shared__ int32_t s_next;  // T at the next sub-segment's start (packed halves)
    const ProbeSeg g = segs[blockIdx.x];
    const ProbeIv I = A.ivs[g.iv];
    const ScanFile& F = A.files[I.file];
    const int64_t n = F.n, B = F.B;
    const uint8_t* __restrict__ data = F.data;
    const int64_t q0 = g.q0, q1 = q0 + g.len;  // every window full: q1 - 1 <= n - B
    const int64_t nb = n - B;
    auto clampB = [&](int64_t p) { return p < nb ? p : nb; };
    // the anchor: T(q0) = (sum x, sum (B - i) x_{q0 + i}) over the window [q0, q0 + B) (full: q0 <= n - B)
    int32_t h[2] = {0, 0};
    range_sums(data, n, q0, q0 + B, q0, h[0], h[1]);
    block_reduce<2>(h, sh);
    uint32_t s1o = (uint32_t)h[0], s2o = (uint32_t)B * (uint32_t)h[0] - (uint32_t)h[1];
    const ProbeTable table{F.slots, F.mask};
    const int nsmall = F.nsmall;
    const int t = threadIdx.x;
    for (int64_t base = q0; base < q1; base += PROBE_LONG_SUB) {
        const int64_t p0 = base + (int64_t)t * PROBE_LONG_PPL;
        int32_t pre[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < PROBE_LONG_PPL / 16; ++k) {  // the lane's bytes at p0 and at p0 + B: its sums
            uint32_t wa[4], wb[4];
            load16(data, n, p0 + 16 * k, wa);
            load16(data, n, p0 + B + 16 * k, wb);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                dword_sums(wa[j], (uint32_t)(p0 + 16 * k + 4 * j - base), pre[0], pre[1]);
                dword_sums(wb[j], (uint32_t)(p0 + B + 16 * k + 4 * j - base), pre[2], pre[3]);
            }
        }
        block_exscan<4>(pre, sh);  // sums over [base, p0) and [base + B, p0 + B), weights j - base
        const bool live = p0 < q1;
        if (live) {
            const uint32_t P1e = s1o + (uint32_t)pre[2];
            const uint32_t P2e = (uint32_t)B * s1o - s2o + (uint32_t)pre[3];
            const uint32_t s1 = P1e - (uint32_t)pre[0];
            const uint32_t s2 = (uint32_t)(p0 + B - base) * s1 - (P2e - (uint32_t)pre[1]);
            const uint32_t ehi = I.e_hi + I.e_lo * (uint32_t)(clampB(p0) - clampB(I.anchor));
            // the rolling value's halves kept apart (each exact mod 2^16: the Java subtract-then-add of
            // Rolling.java:25-60 in two adds each, as the chain walk's tiles), packed into the key per position
            uint32_t u1 = (s1 + I.e_lo) & 0xFFFFu, u2 = (s2 + ehi) & 0xFFFFu;
#pragma unroll 1
            for (int grp = 0; grp < PROBE_LONG_PPL / 16; ++grp) {  // 16 positions at a time (bytes re-read: L1)
                uint32_t wa[4], wb[4];
                load16(data, n, p0 + 16 * grp, wa);
                load16(data, n, p0 + B + 16 * grp, wb);
                uint32_t key[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {  // full windows throughout: w = B, the add always follows
                    key[i] = __builtin_amdgcn_perm(u2, u1, 0x05040100u);  // (u1 & 0xFFFF) | (u2 << 16)
                    const int32_t xo = sbyte_of(wa, i), xi = sbyte_of(wb, i);
                    u1 += (uint32_t)(xi - xo);
                    u2 += u1 - (uint32_t)__mul24((int)B, xo);
                }
                const uint32_t valid = probe_valid16(p0 + 16 * grp, I.a, I.b < q1 ? I.b : q1);
                if (valid) probe_check16(F, table, nsmall, key, valid, p0 + 16 * grp);
            }
            if (t == PROBE_THREADS - 1) {  // R(p0 + 64) less E there: the next sub-segment's anchor T
                const int64_t pn = p0 + PROBE_LONG_PPL;
                const uint32_t en = I.e_hi + I.e_lo * (uint32_t)(clampB(pn) - clampB(I.anchor));
                const uint32_t r = (u1 & 0xFFFFu) | (u2 << 16);
                s_next = (int32_t)((((r & 0xFFFFu) - I.e_lo) & 0xFFFFu) | (((r >> 16) - en) << 16));
            }
        }
        __syncthreads();
        s1o = (uint32_t)s_next & 0xFFFFu;
        s2o = (uint32_t)s_next >> 16;
        __syncthreads();
    }
}

hipError_t launch_probe_long(const ProbeArgs& args, const ProbeSeg* segs, uint32_t nsegs, hipStream_t s) {
    if (nsegs == 0) return hipSuccess;
    hipLaunchKernelGGL(probe_long_kernel, dim3(nsegs), dim3(PROBE_THREADS), 0, s, args, segs);
    return hipGetLastError();
}

hipError_t launch_probe_first(const ProbeArgs& args, uint32_t ntiles, const PartialTile* ptiles, uint32_t nptiles,
                              hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    if (nptiles > 0)
        hipLaunchKernelGGL(probe_partials_kernel, dim3(nptiles), dim3(256), 0, s, args.files, ptiles, args.partials);
    hipLaunchKernelGGL(probe_first_kernel, dim3(ntiles), dim3(PROBE_THREADS), 0, s, args);
    return hipGetLastError();
}


// ------------------------------------------------------------------------------------------------
// The batched flush chain on the device (resolver.h FlushChain; the host form is resolver.cpp flush_chain_host).
// Its recurrence is linear in the desync.  With a_i, b_i the (elo, ehi) after flush i, all mod 2^16:
//   a_i = a_{i-1} + d_i,                       d_i = lo T(f_i) - x_i + add_i y_i - lo T(f_i + B)
//   b_i = b_{i-1} + a_{i-1} D_i + g_i + add_i a_i,  g_i = hi T(f_i) - B x_i - hi T(f_i + B) + add_i lo T(f_i + B)
// x_i, y_i the signed bytes at f_i and f_i + 2B - 1; add_i: s2_i = f_i + B <= last and its window is full (the
// Java code adds the window's new last byte, Sender.java:1308-1310); D_i = min(f_i, n - B) - min(s2_{i-1}, n - B)
// (E_hi's drift over the interval), D_0 = 0; a_{-1} = el, b_{-1} = eh.  Two block scans give every step at once,
// on the device between the round's gathers and its probe, instead of a serial host loop between two round trips.
// One workgroup per chain (K <= 4096: 16 steps per thread).
// ------------------------------------------------------------------------------------------------
constexpr int FCHAIN_THREADS = 256;
__device__ __forceinline__ uint32_t fchain_exscan(uint32_t v, uint32_t* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < FCHAIN_THREADS; o <<= 1) {
        const uint32_t x = t >= o ? sh[t - o] : 0u;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    const uint32_t incl = sh[t];
    __syncthreads();
    return incl - v;
}
__global__ __launch_bounds__(FCHAIN_THREADS) void flush_chain_kernel(const FlushChainJob* __restrict__ jobs) {
    __shared__ uint32_t sh[FCHAIN_THREADS];
    const FlushChainJob J = jobs[blockIdx.x];
    const int per = (J.K + FCHAIN_THREADS - 1) / FCHAIN_THREADS;
    const int i0 = (int)threadIdx.x * per, i1 = min(J.K, i0 + per);
    const int64_t nB = J.n - J.B;
    auto clampB = [&](int64_t p) { return p < nB ? p : nB; };
    // step i's terms (d, g, add, D) from the gathered sums and bytes
    auto terms = [&](int i, uint32_t& d, uint32_t& g, uint32_t& add, uint32_t& D) {
        const int64_t fi = J.f + 10 * J.B * (int64_t)i, s2 = fi + J.B;
        const uint32_t T0 = (uint32_t)J.tv[2 * i], T1 = (uint32_t)J.tv[2 * i + 1];
        const uint32_t x = (uint32_t)(int32_t)(int8_t)J.bv[2 * i];
        add = (s2 <= J.last && (J.n - s2 >= J.B)) ? 1u : 0u;
        const uint32_t y = add ? (uint32_t)(int32_t)(int8_t)J.bv[2 * i + 1] : 0u;
        d = (T0 & 0xFFFFu) - x + y - (T1 & 0xFFFFu);
        g = (T0 >> 16) - (uint32_t)J.B * x - (T1 >> 16) + add * (T1 & 0xFFFFu);
        D = i == 0 ? 0u : (uint32_t)(clampB(fi) - clampB(fi - 9 * J.B));
    };
    uint32_t dsum = 0;
    for (int i = i0; i < i1; ++i) {
        uint32_t d, g, add, D;
        terms(i, d, g, add, D);
        dsum += d;
    }
    const uint32_t a_base = J.el + fchain_exscan(dsum, sh);  // a_{i0 - 1}
    uint32_t a_prev = a_base, hsum = 0;
    for (int i = i0; i < i1; ++i) {
        uint32_t d, g, add, D;
        terms(i, d, g, add, D);
        const uint32_t a = a_prev + d;
        hsum += a_prev * D + g + add * a;
        a_prev = a;
    }
    uint32_t b = J.eh + fchain_exscan(hsum, sh);  // b_{i0 - 1}
    a_prev = a_base;
    for (int i = i0; i < i1; ++i) {
        uint32_t d, g, add, D;
        terms(i, d, g, add, D);
        const uint32_t a = a_prev + d;
        b += a_prev * D + g + add * a;
        a_prev = a;
        J.out[2 * i] = a & 0xFFFFu;
        J.out[2 * i + 1] = b & 0xFFFFu;
        if (i < J.niv) {
            J.iv[i].e_lo = a & 0xFFFFu;
            J.iv[i].e_hi = b & 0xFFFFu;
        }
    }
}

hipError_t launch_flush_chain(const FlushChainJob* jobs, uint32_t njobs, hipStream_t s) {
    if (njobs == 0) return hipSuccess;
    hipLaunchKernelGGL(flush_chain_kernel, dim3(njobs), dim3(FCHAIN_THREADS), 0, s, jobs);
    return hipGetLastError();
}

// A kernel that does nothing: its first launch makes the runtime load this file's code object (the search kernels) --
// 0.6-1.8 ms on a fresh context, which rsh_ctx_create pays instead of the first call (launch_warm).
__global__ void warm_scan_kernel() {}
hipError_t launch_warm_scan(hipStream_t s) {
    hipLaunchKernelGGL(warm_scan_kernel, dim3(1), dim3(64), 0, s);
    return hipGetLastError();
}

}  // namespace rsh
