// device.hip -- gfx950 (CDNA4) kernels for java-rsync's delta-transfer checksum path.
//
// Integer/byte work, HBM-bound (the MD5 chains are VALU work).  The one matrix-core use is the
// production K1's weak sums: two v_mfma_i32_16x16x64_i8 per stage against a 0/1-and-index weight
// matrix (exact int32, see block_sums_pipe_kernel), which takes them off the VALU that MD5 saturates.
// No GEMM reshaping anywhere else.  Layout in HBM: the file is one flat byte array (caller's
// buffer, 256-B aligned from hipMalloc); per-chunk outputs are struct-of-arrays (weak int32[C],
// strong uint8[C*dl]).  See DESIGN.md for the roofline of each kernel.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "device.h"
#include "device_common.h"
#include "md5_core.h"
#include "options.h"

#include <algorithm>
#include <type_traits>

namespace rsh {

// ------------------------------------------------------------------------------------------------
// Weak-sum arithmetic (util/Rolling.java).  For a chunk x[0..L) of signed bytes:
//   s1 = sum x_i,  s2 = sum (L - i) x_i = L*s1 - u,  u = sum i*x_i;  weak = (s1 & 0xFFFF) | (s2 << 16).
// Per 64-byte block at chunk offset `off` the packed signed-byte dot product v_dot4_i32_i8 gives
// a = sum x and b = sum k*x_k (k local, weights <= 63 fit int8), so u += off*a + b.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void weak_block(const uint32_t (&m)[16], int32_t& s1, int32_t& u, uint32_t off) {
    int32_t a = 0, b = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        a = __builtin_amdgcn_sdot4((int)m[j], 0x01010101, a, false);
        const int w = (4 * j) | ((4 * j + 1) << 8) | ((4 * j + 2) << 16) | ((4 * j + 3) << 24);
        b = __builtin_amdgcn_sdot4((int)m[j], w, b, false);
    }
    s1 += a;
    u += (int32_t)(off * (uint32_t)a) + b;
}


// MD5 of one 64-byte block plus its weak-sum contribution at chunk offset `off`.
__device__ __forceinline__ void md5_weak_block(Md5State& st, const uint32_t (&m)[16], int32_t& s1, int32_t& u,
                                               uint32_t off) {
    int32_t a, b;
    md5_compress_weak(st, m, a, b);
    s1 += a;
    u += (int32_t)(off * (uint32_t)a) + b;
}

// Final 1-2 MD5 blocks: r (< 64) trailing data bytes at p, then the 4 seed bytes, 0x80, zero pad and
// the 64-bit bit length of (chunk || seed).  Also folds the r bytes into the weak sums.
__device__ __forceinline__ void md5_tail(Md5State& st, const uint8_t* p, uint32_t r, uint32_t seed,
                                      uint64_t msg_bytes, int32_t& s1, int32_t& u, uint32_t off) {
    for (uint32_t i = 0; i < r; ++i) {
        const int32_t x = sbyte(p[i]);
        s1 += x;
        u += (int32_t)((off + i) * (uint32_t)x);
    }
    const uint64_t bits = msg_bytes * 8;
    const uint32_t nblk = (r + 4 + 9 <= 64) ? 1 : 2;
    for (uint32_t blk = 0; blk < nblk; ++blk) {
        uint32_t m[16];
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = blk * 64 + 4 * w + j;
                uint32_t byte;
                if (i < r) byte = p[i];
                else if (i < r + 4) byte = (seed >> (8 * (i - r))) & 0xFFu;
                else if (i == r + 4) byte = 0x80u;
                else byte = 0;
                if (blk == nblk - 1 && w >= 14) byte = (uint32_t)(bits >> (8 * (4 * (w - 14) + j))) & 0xFFu;
                word |= byte << (8 * j);
            }
            m[w] = word;
        }
        md5_compress(st, m);
    }
}

__device__ __forceinline__ void unpack(const uint4 (&q)[4], uint32_t (&m)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        m[4 * i + 0] = q[i].x;
        m[4 * i + 1] = q[i].y;
        m[4 * i + 2] = q[i].z;
        m[4 * i + 3] = q[i].w;
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
static const int* never_word();

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    const u32x4* v = reinterpret_cast<const u32x4*>(p);
    const u32x4 t = NT ? __builtin_nontemporal_load(v) : *v;
    return make_uint4(t.x, t.y, t.z, t.w);
}

template <int ALIGN, bool NT = true>
__device__ __forceinline__ void load_block(const uint8_t* p, uint4 (&q)[4]) {
    if constexpr (ALIGN == 16) {
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = ld16<NT>(p + 16 * i);
    } else if constexpr (ALIGN == 4) {
        const uint32_t* v = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
    } else if constexpr (ALIGN == 2) {
        // any alignment, wide loads: the 4 or 5 aligned 16-B pieces that hold the 64 bytes, then a per-lane
        // dword select (lanes of one wave may sit at different offsets) and a byte funnel shift; the fifth
        // piece is read only when the block is not 16-B aligned (it holds byte p + 63 then)
        const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
        const u32x4* v = reinterpret_cast<const u32x4*>(pa & ~(uintptr_t)15);
        const uint32_t o = (uint32_t)(pa & 15), wo = o >> 2, sh = o & 3;
        uint32_t d[20];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4 t = v[i];
            d[4 * i] = t.x;
            d[4 * i + 1] = t.y;
            d[4 * i + 2] = t.z;
            d[4 * i + 3] = t.w;
        }
        u32x4 t4 = {0u, 0u, 0u, 0u};
        if (o) t4 = v[4];
        d[16] = t4.x;
        d[17] = t4.y;
        d[18] = t4.z;
        d[19] = t4.w;
        uint32_t e[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) e[i] = wo == 0 ? d[i] : wo == 1 ? d[i + 1] : wo == 2 ? d[i + 2] : d[i + 3];
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sh);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
    } else if constexpr (ALIGN == 0) {
        // any alignment: the 16 or 17 aligned dwords that hold the 64 bytes, funnel-shifted (v_alignbyte_b32);
        // the 17th is read only when the block is not dword aligned, so no byte past p + 63's dword is touched
        const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
        const uint32_t* v = reinterpret_cast<const uint32_t*>(pa & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(pa & 3);
        uint32_t d[17];
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = v[i];
        d[16] = sh ? v[16] : 0u;
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
    } else {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
                   ((uint32_t)p[4 * i + 3] << 24);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
    }
}

// ------------------------------------------------------------------------------------------------
// K1: Generator block sums.  One lane = one chunk (MD5 is a serial chain per message, so the chunk is
// the unit of parallelism); each lane streams its chunk 64 B at a time with a PF-deep register ring
// of in-flight loads so HBM latency hides behind the MD5 rounds of the blocks already loaded.
// ------------------------------------------------------------------------------------------------
template <int ALIGN, int PF, bool NT = true>
__device__ __forceinline__ void lane_chunk_sums(const uint8_t* __restrict__ data, int64_t n, uint32_t B, uint32_t c,
                                                uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
                                                uint8_t* __restrict__ strong_out) {
    const int64_t base = (int64_t)c * B;
    const int64_t rem = n - base;
    const uint32_t L = rem < (int64_t)B ? (uint32_t)rem : B;
    const uint8_t* p = data + base;
    const uint32_t nfull = L >> 6;

    Md5State st = md5_init();
    int32_t s1 = 0, u = 0;
    uint4 q[PF][4];
#pragma unroll
    for (int j = 0; j < PF; ++j)
        if ((uint32_t)j < nfull) load_block<ALIGN, NT>(p + 64 * j, q[j]);

    uint32_t i = 0;
    // Steady state: every consumed slot is refilled PF blocks ahead, unconditionally.
    for (; i + 2 * PF <= nfull; i += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            uint32_t m[16];
            unpack(q[j], m);
            load_block<ALIGN, NT>(p + 64 * (size_t)(i + j + PF), q[j]);
            weak_block(m, s1, u, 64 * (i + j));
            md5_compress(st, m);
        }
    }
    // Drain: fewer than 2*PF blocks remain.
    for (; i < nfull; i += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const uint32_t blk = i + j;
            if (blk < nfull) {
                uint32_t m[16];
                unpack(q[j], m);
                if (blk + PF < nfull) load_block<ALIGN, NT>(p + 64 * (size_t)(blk + PF), q[j]);
                weak_block(m, s1, u, 64 * blk);
                md5_compress(st, m);
            }
        }
    }
    md5_tail(st, p + 64 * (size_t)nfull, L & 63u, seed, (uint64_t)L + 4, s1, u, 64 * nfull);

    const int32_t s2 = (int32_t)(L * (uint32_t)s1 - (uint32_t)u);
    weak_out[c] = (int32_t)(((uint32_t)s1 & 0xFFFFu) | ((uint32_t)s2 << 16));
    store_digest(strong_out + (size_t)c * dl, st, dl);
}

template <int ALIGN, int PF, bool NT = true>
__global__ __launch_bounds__(64) void block_sums_kernel(const uint8_t* __restrict__ data, int64_t n, uint32_t B,
                                                        uint32_t nchunks, uint32_t dl, uint32_t seed,
                                                        int32_t* __restrict__ weak_out,
                                                        uint8_t* __restrict__ strong_out, uint32_t c_first) {
    const uint32_t c = c_first + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    lane_chunk_sums<ALIGN, PF, NT>(data, n, B, c, dl, seed, weak_out, strong_out);
}

// Batched files, one lane per chunk: wave w takes chunks [c_first, c_first + 64) of lanes[w]'s file.
template <int ALIGN>
__global__ __launch_bounds__(64) void block_sums_lane_batch_kernel(const K1Lane* __restrict__ lanes, uint32_t seed) {
    const K1Lane e = lanes[blockIdx.x];
    const uint32_t c = e.c_first + threadIdx.x;
    if (c >= e.nchunks) return;
    // byte-aligned files read through the funnel-shift form (ALIGN 0), 4 blocks ahead
    lane_chunk_sums<ALIGN == 1 ? 0 : ALIGN, ALIGN == 16 ? 4 : ALIGN == 4 ? 2 : 4, ALIGN != 1>(e.data, e.n, e.B, c, e.dl,
                                                                                          seed, e.weak, e.strong);
}

typedef int v4i32 __attribute__((ext_vector_type(4)));

// Weak sums on the matrix pipe: see block_sums_pipe_body (weak_words).  Until round 5 the shift kernel summed whole
// 128-B LDS lines per group of 16 chunks (C_g += W_h x X_{g,h}, a permuted column order against bank conflicts;
// DESIGN.md sec. 4); since round 6 it uses the pipelined kernel's form as well.

// ABORT (the Sender's speculation only): every 16 stages the wave reads *abort_flag (uncached device
// memory, set by a stream write-value packet) with a cache-bypassing scalar load and exits when it
// equals abort_gen -- the resolver finished without needing this launch's results.  The read waits
// for itself only (the LDS traffic of the iteration is consumed by then; vector loads are untouched).
__device__ __forceinline__ int poll_abort(const int* flag) {
    int v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(flag));
    return v;
}

// ------------------------------------------------------------------------------------------------
// K1, software-pipelined (production).  One wave owns 64 consecutive full-length chunks (L = B, B % 128 == 0).
// A stage is the next 128 B of every chunk: 8 buffer loads per lane, each instruction reading 8 whole 128-B lines
// (8 lanes per line) instead of 64 scattered 16-B pieces; the wave transposes the stage through LDS (row = 8 data
// slots + 1 pad slot, so the 8-lane ds_write_b128 and the 16-lane ds_read_b128 groups are bank-conflict free) and
// each lane then runs its chunk's MD5 over the two 64-B blocks, one lane = one chunk.  No LDS round trip ever sits
// on a wave's critical path: stage s+1 is written to the second LDS
// buffer at the top of stage s, its message words and MFMA operands are read back into registers
// between the two MD5 blocks of stage s, so they have landed long before stage s+1 starts.  The weak-sum
// MFMAs of stage s sit between its MD5 blocks too.  Two stages of loads stay in flight (slots q[0..1]).
// LDS operations of one wave execute in order, so a compiler-only barrier orders the write and the
// reads of a buffer; no s_waitcnt lgkmcnt(0) / s_barrier per stage.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// The production MD5 step form (md5_asm.inc: 16 steps per asm statement, no s_nop after the rotates; kbench
// A/Bs of the other forms in DESIGN.md sec. 4)
__device__ __forceinline__ void md5_stream_block(Md5State& st, const uint32_t (&m)[16]) { md5_compress_rot16n(st, m); }

// amdgpu_num_vgpr(192): two waves fill 384 of a SIMD's 512 registers, leaving room for one wave of the
// resolver's range probe (104) to run beside the Sender's speculation launch in head mode.
// MULTI (batched files, K1Group per wave): the wave's 64 chunks, B, dl and output slots come from
// groups[blockIdx.x] instead of (data, B, dl, weak_out, strong_out) + blockIdx.x * 64 chunks.
// K1_PIPE_ATTR (A/B at build time, -DRSH_K1_NUMVGPR=N): the register budget.  waves_per_eu(3) caps the
// kernel at 168 VGPRs, which spills 12 of them to scratch (20 B/lane); num_vgpr(N) with N >= 184 does not.
#ifndef RSH_K1_TAIL_PF
#define RSH_K1_TAIL_PF 2
#endif
#ifdef RSH_K1_NUMVGPR
#define K1_PIPE_ATTR __attribute__((amdgpu_num_vgpr(RSH_K1_NUMVGPR)))
#else
#define K1_PIPE_ATTR __attribute__((amdgpu_waves_per_eu(3)))
#endif
// GATHER (leftover chunks of a launch): the wave's gcnt <= 64 chunks are full-length chunks at any base,
// loaded with plain dwordx4 loads (16-B aligned or not) from one 64-bit pointer per 8-chunk row instead of a
// buffer descriptor.  gt != nullptr: chunk i is gt[i] (K1Tail: any file; the segmented launch); else chunk i
// is data + i B with outputs weak_out[i], strong_out[i dl] (a single launch's partial last wave).  Lanes past
// gcnt digest chunk 0 again and store nothing.
// Weak sums (since round 4): the weak sums from the MD5 message words already in registers instead of a second read of
// the stage from LDS in the MFMA operand layout: per 64-B block, four v_mfma_i32_16x16x64_i8 with B = the lane's
// own 16-byte quarter w of its block and A = rows that select one lane group each (row m reads lane group m & 3:
// type m >> 2 = 0 ones, 1 the byte's offset 16 w + i in the block), all into one accumulator -- chunk n + 16 q's
// block sum lands in lane n (element q), its weighted sum in lane n + 16.  Saves the 8 ds_read_b128 per stage: the
// same cycles at a higher clock, 2.5 % less time (kbench A/B, profiles/r4/r4e_kbench_weakw_k3s*).
// ABORT: the wave polls *abort_flag (never_word() when the launch has no abort word of its own).
// WEAKV (kbench A/B only, variant 1010): the weak sums on the VALU (weak_block: 32 v_dot4_i32_i8 per 64-B block)
// instead of the matrix pipe -- the form that drops the MFMAs' power for 8 % more VALU issue.
template <bool MULTI = false, bool GATHER = false, bool WEAKV = false>
__device__ __forceinline__ void block_sums_pipe_body(const uint8_t* __restrict__ data, uint32_t B, uint32_t dl,
                                                             uint32_t seed, int32_t* __restrict__ weak_out,
                                                             uint8_t* __restrict__ strong_out,
                                                             const int* abort_flag = nullptr, int abort_gen = 0,
                                                             const K1Group* __restrict__ groups = nullptr,
                                                             int64_t n = 0, uint32_t nchunks = 0,
                                                             uint32_t main_waves = 0xFFFFFFFFu,
                                                             const K1Tail* __restrict__ gt = nullptr,
                                                             uint32_t gcnt = 0, uint32_t gsel = 0xFFFFFFFFu) {
    constexpr int ROW = 9;
    constexpr int BUF = 64 * ROW;  // uint4 slots per LDS buffer
    constexpr int TAIL_PF = RSH_K1_TAIL_PF;
    if constexpr (!MULTI && !GATHER) {
        // tail waves (blockIdx >= main_waves): one lane per chunk left over (a partial last wave, the short last
        // chunk), dispatched with the main waves rather than as a launch queued behind them (a lone wave takes
        // as long as one lane's window: 1.9 ms at B = 128 KiB).  Plain dwordx4 loads at the lane's own address,
        // 16-B aligned or not (gfx950 serves unaligned vector loads; bit-exact at every offset, tests): kbench,
        // 16 GiB of per-lane waves at B = 128 KiB, 3.6 ms with plain loads against 7.7 ms non-temporal and
        // 4.7 ms funnel-shifting 17 dword loads per block (one wave alone: 1.6 ms, the coalesced kernel 1.9).
        if (blockIdx.x >= main_waves) {
            const uint32_t c = main_waves * 64u + (blockIdx.x - main_waves) * 64u + threadIdx.x;
            if (c < nchunks) lane_chunk_sums<16, TAIL_PF, false>(data, n, B, c, dl, seed, weak_out, strong_out);
            return;
        }
    }
    asm volatile("; occupancy pin" ::: "v175");  // at most 2 waves per SIMD
    extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // 2 buffers (sized at launch)
    const int l = threadIdx.x;
    uint32_t c0 = blockIdx.x * 64u;
    const uint8_t* gdata = data + (size_t)c0 * B;
    if constexpr (MULTI) {
        const K1Group g = groups[gsel == 0xFFFFFFFFu ? blockIdx.x : gsel];  // gsel: a persistent wave's group
        gdata = g.data;
        B = g.B;
        dl = g.dl;
        weak_out = g.weak;
        strong_out = g.strong;
        c0 = 0;
        if (g.abort) abort_flag = g.abort;  // per-file cancellation (batched Sender speculation)
    }
    [[maybe_unused]] const uint8_t* rp[8];  // GATHER: row j's lane address (chunk (l >> 3) + 8 j, piece l & 7)
    if constexpr (GATHER) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t ci = (uint32_t)(l >> 3) + 8u * (uint32_t)j;
            const uint32_t cs = ci < gcnt ? ci : 0u;
            if (gt) {
                const K1Tail t = gt[cs];
                rp[j] = t.data + (size_t)t.c * B + 16u * (uint32_t)(l & 7);
            } else {
                rp[j] = data + (size_t)cs * B + 16u * (uint32_t)(l & 7);
            }
        }
        c0 = 0;
    }
    const uint32_t nst = B >> 7;  // host guarantees nst >= 4
    const int wr0 = (l >> 3) * ROW + (l & 7);
    const int rd0 = l * ROW;

    v4i32 wW[4];  // the A operand for block quarter w
    v4i32 accW = {0, 0, 0, 0}, RW = {0, 0, 0, 0};
    {
        const int m = l & 15, q = l >> 4, type = m >> 2;
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t word = 0;
                if (q == (m & 3) && type == 0) word = 0x01010101u;
                else if (q == (m & 3) && type == 1)
#pragma unroll
                    for (int b = 0; b < 4; ++b) word |= (uint32_t)(16 * w + 4 * d + b) << (8 * b);
                wW[w][d] = (int)word;
            }
    }

    uint4 q[2][8];  // load slots: stage s+1 and s+2 in flight while stage s computes
    uint4 Wa[4];    // words of the current stage's block 0 (then: the next stage's block 0)
    uint4 Wb[4];    // words of the current stage's block 1
    // Buffer loads: the wave's 64 chunks (64 * B <= 8 MiB) behind one descriptor, a 32-bit lane offset and
    // a scalar offset per 8-chunk row j -- one VGPR of addressing instead of eight 64-bit pointers.
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(gdata), 0, (int)(64 * B), 0x00020000);
    const uint32_t lane_off = (uint32_t)(l >> 3) * B + 16u * (uint32_t)(l & 7);
    auto load = [&](uint4 (&dst)[8], uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (GATHER) {
                dst[j] = ld16<false>(rp[j] + 128u * stg);
            } else {
                const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane_off + 128u * stg, (int)(j * 8u * B), 2);
                dst[j] = make_uint4(t.x, t.y, t.z, t.w);
            }
        }
    };
    auto put = [&](const uint4 (&src)[8], int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds_all[buf * BUF + wr0 + j * 8 * ROW] = src[j];
    };
    auto get_words = [&](uint4 (&w)[4], int buf, int h) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = lds_all[buf * BUF + rd0 + 4 * h + k];
    };
    Md5State st = md5_init();
    auto md5_block = [&](const uint4 (&w)[4]) __attribute__((always_inline)) {
        uint32_t m[16];
        unpack(w, m);
        md5_stream_block(st, m);
    };
    [[maybe_unused]] int32_t vs1 = 0, vu = 0;  // WEAKV: the lane's own sums
    auto weak_words = [&](const uint4 (&w)[4], [[maybe_unused]] uint32_t off) __attribute__((always_inline)) {
        if constexpr (WEAKV) {  // one 64-B block at chunk offset off
            uint32_t m[16];
            unpack(w, m);
            weak_block(m, vs1, vu, off);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) RW[e] += accW[e];  // R += P_{b-1}
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const v4i32 b4 = {(int)w[k].x, (int)w[k].y, (int)w[k].z, (int)w[k].w};
                accW = __builtin_amdgcn_mfma_i32_16x16x64_i8(wW[k], b4, accW, 0, 0, 0);
            }
        }
    };
    // One stage with compile-time parity P: LDS buffer P holds it, q[P ^ 1] the next stage's data.
    // Block-1 words are read at the top (they land during block 0); the next stage's block-0 words are read
    // between the blocks (they land during block 1).
    auto stage = [&](auto pc, uint32_t si, bool has_next, bool refill) __attribute__((always_inline)) {
        constexpr int P = decltype(pc)::value;
        if (has_next) {
            put(q[P ^ 1], P ^ 1);
            if (refill) load(q[P ^ 1], si + 3);
        }
        get_words(Wb, P, 1);
        md5_block(Wa);
        weak_words(Wa, 128u * si);
        compiler_fence();
        if (has_next) get_words(Wa, P ^ 1, 0);
        md5_block(Wb);
        weak_words(Wb, 128u * si + 64u);
        compiler_fence();
    };

    load(q[0], 0);
    load(q[1], 1);
    if constexpr (MULTI) {  // a group whose file was resolved before the wave started does nothing
        int f0;
        asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(f0) : "s"(abort_flag));
        if (f0 == abort_gen) return;
    }
    put(q[0], 0);
    load(q[0], 2);
    compiler_fence();
    get_words(Wa, 0, 0);
    uint32_t s = 0;
    // steady state: every stage has a next stage and a refill (branch-free: exact vmcnt bookkeeping)
    // Abort: one scalar load (glc: from L2, not the scalar cache) of the abort word per 2 stages, issued at
    // the top of the iteration and compared at the bottom, so its latency hides behind the two stages.
    // The compiler does not see the load; its own lgkmcnt(N) waits for LDS stay safe with one extra
    // operation in flight (they only get stricter).
    int flag = 0;
    for (; s + 5 <= nst && flag != abort_gen; s += 2) {
        asm volatile("s_load_dword %0, %1, 0x0 glc" : "=s"(flag) : "s"(abort_flag));
        stage(std::integral_constant<int, 0>{}, s, true, true);
        stage(std::integral_constant<int, 1>{}, s + 1, true, true);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(flag));
    }
    if (flag == abort_gen) return;
    for (; s < nst; s += 2) {  // drain
        stage(std::integral_constant<int, 0>{}, s, s + 1 < nst, s + 3 < nst);
        if (s + 1 < nst) stage(std::integral_constant<int, 1>{}, s + 1, s + 2 < nst, s + 4 < nst);
    }
    {
        const uint64_t bits = ((uint64_t)B + 4) * 8;
        uint32_t m[16] = {seed, 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, (uint32_t)bits, (uint32_t)(bits >> 32)};
        md5_compress(st, m);
    }
    int32_t s1, u;
    if constexpr (WEAKV) {
        s1 = vs1;
        u = vu;
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) RW[e] += accW[e];
        const int n = l & 15, q = l >> 4;
        int32_t tS[4], tR[4], tW[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            tS[e] = __shfl(accW[e], n, 64);
            tR[e] = __shfl(RW[e], n, 64);
            tW[e] = __shfl(accW[e], n + 16, 64);
        }
        const int32_t S = q == 0 ? tS[0] : q == 1 ? tS[1] : q == 2 ? tS[2] : tS[3];
        const int32_t Rq = q == 0 ? tR[0] : q == 1 ? tR[1] : q == 2 ? tR[2] : tR[3];
        const int32_t Wq = q == 0 ? tW[0] : q == 1 ? tW[1] : q == 2 ? tW[2] : tW[3];
        s1 = S;
        u = (int32_t)(64u * (2u * nst * (uint32_t)S - (uint32_t)Rq)) + Wq;
    }
    uint32_t c = c0 + l;
    if constexpr (GATHER) {
        if ((uint32_t)l >= gcnt) return;
        if (gt) {
            const K1Tail t = gt[l];
            weak_out = t.weak;
            strong_out = t.strong;
            c = t.c;
        }
    }
    const int32_t s2 = (int32_t)(B * (uint32_t)s1 - (uint32_t)u);
    weak_out[c] = (int32_t)(((uint32_t)s1 & 0xFFFFu) | ((uint32_t)s2 << 16));
    store_digest(strong_out + (size_t)c * dl, st, dl);
}

template <bool MULTI = false>
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_kernel(const uint8_t* __restrict__ data, uint32_t B, uint32_t dl,
                                                             uint32_t seed, int32_t* __restrict__ weak_out,
                                                             uint8_t* __restrict__ strong_out,
                                                             const int* abort_flag = nullptr, int abort_gen = 0,
                                                             const K1Group* __restrict__ groups = nullptr,
                                                             int64_t n = 0, uint32_t nchunks = 0,
                                                             uint32_t main_waves = 0xFFFFFFFFu) {
    block_sums_pipe_body<MULTI>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen, groups, n, nchunks,
                                main_waves);
}
// The production K1 with the partial last wave's full-length chunks as a gathered coalesced wave (the tail
// waves past main_waves: ceil(tail_full / 64) gathered ones, then the short last chunk, if any, per lane).  A
// per-lane wave runs ~20% slower than a coalesced one and, when every wave runs in the first round, sets the
// launch's end.  Used only for launches with such a tail: the exact-multiple launches keep
// block_sums_pipe_kernel.  Its register budget is 256 (2 waves/SIMD): under K1_PIPE_ATTR the two bodies spill.
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(256))) void block_sums_pipe_tailg_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen, int64_t n, uint32_t nchunks,
    uint32_t main_waves, uint32_t tail_full) {
    if (blockIdx.x >= main_waves) {
        const uint32_t tw = blockIdx.x - main_waves, ngw = (tail_full + 63u) / 64u;
        if (tw < ngw) {
            const uint32_t first = main_waves * 64u + 64u * tw;
            block_sums_pipe_body<false, true>(
                data + (size_t)first * B, B, dl, seed, weak_out + first, strong_out + (size_t)first * dl, abort_flag,
                abort_gen, nullptr, 0, 0, 0xFFFFFFFFu, nullptr, min(64u, tail_full - 64u * tw));
            return;
        }
        const uint32_t c = main_waves * 64u + tail_full + (tw - ngw) * 64u + threadIdx.x;
        if (c < nchunks) lane_chunk_sums<16, RSH_K1_TAIL_PF, false>(data, n, B, c, dl, seed, weak_out, strong_out);
        return;
    }
    block_sums_pipe_body<false>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen, nullptr, n, nchunks,
                                main_waves);
}
bool tail_gather_on() { return opt(OPT_K1_GATHER) != 0; }  // 0: leftover chunks one per lane (options.h)
#ifdef RSH_KBENCH
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_weakv_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen) {
    block_sums_pipe_body<false, false, true>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen);
}
#endif

// Diagnostic (rsh_debug_k1_clock, MI355X_MICROARCH.md "DVFS give-back" item 6): the Generator's production K1 body
// with each wave's shader-clock (s_memtime) and 100 MHz (s_memrealtime) ticks stamped around it and summed over the
// launch; their quotient x 100 MHz is the clock the chip held under this load.  Only this instantiation stamps: the
// production kernels never execute a stamp.  Whole coalesced waves only (n = 64 k B, B % 128 == 0).
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_clock_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen, int64_t n, uint32_t nchunks,
    unsigned long long* __restrict__ clk) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    block_sums_pipe_body<false>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen, nullptr, n, nchunks,
                                0xFFFFFFFFu);
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        atomicAdd(&clk[0], (unsigned long long)(c1 - c0));
        atomicAdd(&clk[1], (unsigned long long)(r1 - r0));
    }
}

hipError_t launch_k1_clock(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t dl, uint32_t seed_word,
                           int32_t* d_weak, uint8_t* d_strong, unsigned long long* d_clk, hipStream_t s) {
    if (B == 0 || B % 128 != 0 || n <= 0 || n % (64 * (int64_t)B) != 0 || dl > 16) return hipErrorInvalidValue;
    const uint32_t nchunks = (uint32_t)(n / B), waves = nchunks / 64;
    const size_t wave_lds = 64 * 9 * sizeof(uint4);
    hipLaunchKernelGGL(block_sums_pipe_clock_kernel, dim3(waves), dim3(64), 2 * wave_lds, s, d_data, B, dl, seed_word,
                       d_weak, d_strong, never_word(), -1, n, nchunks, d_clk);
    return hipGetLastError();
}
#ifndef RSH_K1_SHIFT_VGPR
#define RSH_K1_SHIFT_VGPR 256  // 2 waves/SIMD (the LDS ring and the MFMA tiles of the aligned kernel, plus the funnel)
#endif
// ------------------------------------------------------------------------------------------------
// K1 at a base that is not 128-B aligned.  The Sender's phase-shifted speculation runs K1 over src + s0 for
// any s0; the pipelined kernel's dwordx4 loads at such a base straddle 128-B lines (every 8-lane row touches
// two) and ran at 0.6x of the aligned rate (kbench, 16 GiB at B = 128 KiB: 4.95 ms at offsets 1 and 8 against
// 3.0 ms).  Here every load stays line-aligned: line u of a chunk is its bytes [128u - a, 128u - a + 128),
// a = base % 128, read from base - a; a chunk spans lines 0..nst.
//  * LDS: each chunk row is a two-line ring (16 slots + 1 pad slot), line u in half u & 1.
//  * MD5 stage t (chunk bytes [128t, 128t + 128)) is ring bytes [(128t + a) mod 256, +128): lines t and t + 1,
//    so MD5 runs one step behind the loads.  Step u writes line u + 1 only after reading stage u - 1's
//    block-1 words (lines u - 1 and u; a wave's LDS operations execute in order).  A block's words come from
//    5 slots at slot offset a >> 4 (mod 16) and are funnel-shifted by a & 15 bytes: dword offset
//    W = (a >> 2) & 3 (template), byte shift a & 3 (v_alignbyte_b32).
//  * Weak sums (round 6): from the funnel-shifted MD5 words in registers, in the aligned kernel's form (four MFMAs
//    per 64-B block, block_sums_pipe_body's weak_words).  Until round 5 the MFMAs summed whole LDS lines read a
//    second time in the operand layout (8 ds_read_b128 per line) and took the bytes outside the chunk out per lane;
//    the two forms measured the same (3.32 against 3.32-3.34 ms for 16 GiB at offset 1, profiles/r6/r6u2), this one
//    with 209 VGPRs instead of 235.  So did unaligned ds_read_b128 instead of the funnel: slower (3.70-4.08 ms; the
//    LDS's unaligned reads cost more than the 16 half-rate v_alignbyte_b32 per block, ~4 % of the kernel's time).
//  * Tail waves (blockIdx >= main_waves): one lane per remaining chunk on the per-lane path (any alignment),
//    dispatched with the main waves rather than as a second launch queued behind them.
// ------------------------------------------------------------------------------------------------
// One wave of the shift kernel: 64 full chunks whose first byte is gdata + a (gdata 128-B aligned; the host
// checked [gdata, gdata + 64 B + 128) lies in the data's allocation); weak_out / strong_out point at the
// wave's chunk 0.
template <int W>
__device__ __forceinline__ void shift_wave(const uint8_t* __restrict__ gdata, uint32_t a, uint32_t B, uint32_t dl,
                                           uint32_t seed, int32_t* __restrict__ weak_out,
                                           uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen) {
    constexpr int ROW = 17;
    extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // 64 rows of ROW slots
    const int l = threadIdx.x;
    const uint32_t nst = B >> 7;  // host guarantees 4 <= nst <= 1024
    const uint32_t Q = a >> 4, r = a & 3;
    const int wr0 = (l >> 3) * ROW + (l & 7);
    const int row = l * ROW;

    v4i32 wW[4];  // the A operand for block quarter w (block_sums_pipe_body)
    v4i32 accW = {0, 0, 0, 0}, RW = {0, 0, 0, 0};
    {
        const int m = l & 15, q = l >> 4, type = m >> 2;
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t word = 0;
                if (q == (m & 3) && type == 0) word = 0x01010101u;
                else if (q == (m & 3) && type == 1)
#pragma unroll
                    for (int b = 0; b < 4; ++b) word |= (uint32_t)(16 * w + 4 * d + b) << (8 * b);
                wW[w][d] = (int)word;
            }
    }
    uint4 q[2][8];  // line u + 1 and u + 2 in flight while step u computes
    uint4 Wa[5];    // block 0 of the next MD5 stage
    uint4 Wb[5];    // block 1 of the current MD5 stage
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(gdata), 0, (int)(64 * B + 128), 0x00020000);
    const uint32_t lane_off = (uint32_t)(l >> 3) * B + 16u * (uint32_t)(l & 7);
    auto load = [&](uint4 (&dst)[8], uint32_t line) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane_off + 128u * line, (int)(j * 8u * B), 2);
            dst[j] = make_uint4(t.x, t.y, t.z, t.w);
        }
    };
    auto put = [&](const uint4 (&src)[8], int half) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds_all[wr0 + j * 8 * ROW + 8 * half] = src[j];
    };
    // the 5 slots holding block h of the MD5 stage with parity P (ring offset 128 P + a + 64 h)
    auto get_words = [&](uint4 (&w)[5], int P, int h) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 5; ++k) w[k] = lds_all[row + ((8 * P + 4 * h + Q + k) & 15)];
    };
    Md5State st = md5_init();
    auto md5_block = [&](const uint4 (&w)[5]) __attribute__((always_inline)) {
        uint32_t d[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            d[4 * k] = w[k].x;
            d[4 * k + 1] = w[k].y;
            d[4 * k + 2] = w[k].z;
            d[4 * k + 3] = w[k].w;
        }
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = __builtin_amdgcn_alignbyte(d[W + i + 1], d[W + i], r);
        md5_stream_block(st, m);
        // the block's weak-sum MFMAs (R += P_{b-1} first), as block_sums_pipe_body's weak_words
#pragma unroll
        for (int e = 0; e < 4; ++e) RW[e] += accW[e];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const v4i32 b4 = {(int)m[4 * k], (int)m[4 * k + 1], (int)m[4 * k + 2], (int)m[4 * k + 3]};
            accW = __builtin_amdgcn_mfma_i32_16x16x64_i8(wW[k], b4, accW, 0, 0, 0);
        }
    };
    // Step u: line u sits in half P = u & 1.  PREV: MD5 of stage u - 1; NEXT: write line u + 1 (half P ^ 1) and
    // read the next stage's block 0; REFILL: load line u + 3 into the slot line u + 1 leaves.
    auto step = [&](auto pc, uint32_t u, bool prev, bool next, bool refill) __attribute__((always_inline)) {
        constexpr int P = decltype(pc)::value;
        if (prev) get_words(Wb, P ^ 1, 1);  // lines u - 1 and u, before line u + 1 replaces line u - 1
        compiler_fence();
        if (next) {
            put(q[P ^ 1], P ^ 1);
            if (refill) load(q[P ^ 1], u + 3);
        }
        if (prev) md5_block(Wa);
        compiler_fence();
        if (next) get_words(Wa, P, 0);  // lines u and u + 1
        if (prev) md5_block(Wb);
        compiler_fence();
    };

    load(q[0], 0);
    load(q[1], 1);
    put(q[0], 0);
    load(q[0], 2);
    compiler_fence();
    step(std::integral_constant<int, 0>{}, 0, false, true, true);
    uint32_t u = 1;
    [[maybe_unused]] int flag = 0;
    // steady state: both steps write a line and refill (u + 4 <= nst); abort word polled as in the pipelined K1
    for (; u + 4 <= nst && flag != abort_gen; u += 2) {
        asm volatile("s_load_dword %0, %1, 0x0 glc" : "=s"(flag) : "s"(abort_flag));
        step(std::integral_constant<int, 1>{}, u, true, true, true);
        step(std::integral_constant<int, 0>{}, u + 1, true, true, true);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(flag));
    }
    if (flag == abort_gen) return;
    for (; u <= nst; u += 2) {  // drain: steps up to nst (line nst; MD5 of stage nst - 1)
        step(std::integral_constant<int, 1>{}, u, true, u < nst, u + 3 <= nst);
        if (u + 1 <= nst) step(std::integral_constant<int, 0>{}, u + 1, true, u + 1 < nst, u + 4 <= nst);
    }
    {
        const uint64_t bits = ((uint64_t)B + 4) * 8;
        uint32_t m[16] = {seed, 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, (uint32_t)bits, (uint32_t)(bits >> 32)};
        md5_compress(st, m);
    }
    // as block_sums_pipe_body: chunk n + 16 q's sums in lane n (element q) and lane n + 16
#pragma unroll
    for (int e = 0; e < 4; ++e) RW[e] += accW[e];
    const int n = l & 15, qq = l >> 4;
    int32_t tS[4], tR[4], tW[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        tS[e] = __shfl(accW[e], n, 64);
        tR[e] = __shfl(RW[e], n, 64);
        tW[e] = __shfl(accW[e], n + 16, 64);
    }
    const int32_t S = qq == 0 ? tS[0] : qq == 1 ? tS[1] : qq == 2 ? tS[2] : tS[3];
    const int32_t Rq = qq == 0 ? tR[0] : qq == 1 ? tR[1] : qq == 2 ? tR[2] : tR[3];
    const int32_t Wq = qq == 0 ? tW[0] : qq == 1 ? tW[1] : qq == 2 ? tW[2] : tW[3];
    const int32_t uw = (int32_t)(64u * (2u * nst * (uint32_t)S - (uint32_t)Rq)) + Wq;
    const int32_t s2 = (int32_t)(B * (uint32_t)S - (uint32_t)uw);
    weak_out[l] = (int32_t)(((uint32_t)S & 0xFFFFu) | ((uint32_t)s2 << 16));
    store_digest(strong_out + (size_t)l * dl, st, dl);
}

template <int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(RSH_K1_SHIFT_VGPR))) void block_sums_shift_kernel(
    const uint8_t* __restrict__ data, int64_t n, uint32_t a, uint32_t B, uint32_t nchunks, uint32_t main_waves,
    uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out, uint8_t* __restrict__ strong_out,
    const int* abort_flag, int abort_gen, uint32_t tail_full) {
    if (blockIdx.x >= main_waves) {
        // the first tail_full leftover chunks (full length) as gathered coalesced waves, the rest per lane
        const uint32_t tw = blockIdx.x - main_waves, ngw = (tail_full + 63u) / 64u;
        if (tw < ngw) {
            const uint32_t first = main_waves * 64u + 64u * tw;
            block_sums_pipe_body<false, true>(
                data + (size_t)first * B, B, dl, seed, weak_out + first, strong_out + (size_t)first * dl, abort_flag,
                abort_gen, nullptr, 0, 0, 0xFFFFFFFFu, nullptr, min(64u, tail_full - 64u * tw));
            return;
        }
        const uint32_t c = main_waves * 64u + tail_full + (tw - ngw) * 64u + threadIdx.x;
        if (c < nchunks) lane_chunk_sums<16, 4, false>(data, n, B, c, dl, seed, weak_out, strong_out);
        return;
    }
    const uint32_t c0 = blockIdx.x * 64u;
    shift_wave<W>(data - a + (size_t)c0 * B, a, B, dl, seed, weak_out + c0, strong_out + (size_t)c0 * dl, abort_flag,
                  abort_gen);
}

// Segmented K1: the waves of several chunk sets at different bases in one launch (the Sender's prefix
// speculation at phase 0 and its phase-shifted speculation after an edit: separate launches would need one
// wave more than the chip's 2048 wave slots, and the last wave would start only when another finished).
// Waves [0, nseg) take a K1Seg each (64 full chunks; the dword offset W of its base chosen per wave);
// waves past them take the K1Tail list (the segments' leftover chunks): its first `ngf` entries (full-length
// chunks at any base) 64 to a gathered coalesced wave (block_sums_pipe_body<.., GATHER>), the rest one chunk
// per lane.  A per-lane wave runs ~20% slower than a coalesced one (its loads and v_dot4 weak sums), and as
// the launch's last wave it set the launch's end: kbench, 2047 segment waves + one per-lane wave of 64
// chunks 3.70-3.75 ms against 3.33 ms without it.  Leftover lanes read through the funnel-shift form (dword
// loads at any base; kbench: ahead of wide aligned loads + a per-lane select and of plain unaligned dwordx4).
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(RSH_K1_SHIFT_VGPR))) void block_sums_seg_kernel(
    const K1Seg* __restrict__ segs, uint32_t nseg, const K1Tail* __restrict__ tails, uint32_t ntail, uint32_t B,
    uint32_t dl, uint32_t seed, uint32_t ngf, const int* never) {
    if (blockIdx.x >= nseg) {
        const uint32_t tw = blockIdx.x - nseg, ngw = (ngf + 63u) / 64u;
        if (tw < ngw) {
            block_sums_pipe_body<false, true>(nullptr, B, dl, seed, nullptr, nullptr, never, -1,
                                                               nullptr, 0, 0, 0xFFFFFFFFu, tails + 64u * tw,
                                                               min(64u, ngf - 64u * tw));
            return;
        }
        const uint32_t i = ngf + (tw - ngw) * 64u + threadIdx.x;
        if (i < ntail) {
            const K1Tail t = tails[i];
            lane_chunk_sums<0, 4, false>(t.data, t.n, B, t.c, dl, seed, t.weak, t.strong);
        }
        return;
    }
    const K1Seg g = segs[blockIdx.x];
    switch ((g.a >> 2) & 3) {
        case 0: shift_wave<0>(g.lines, g.a, B, dl, seed, g.weak, g.strong, g.abort, g.abort_gen); break;
        case 1: shift_wave<1>(g.lines, g.a, B, dl, seed, g.weak, g.strong, g.abort, g.abort_gen); break;
        case 2: shift_wave<2>(g.lines, g.a, B, dl, seed, g.weak, g.strong, g.abort, g.abort_gen); break;
        default: shift_wave<3>(g.lines, g.a, B, dl, seed, g.weak, g.strong, g.abort, g.abort_gen);
    }
}

hipError_t launch_block_sums_segments(const K1Seg* d_segs, uint32_t nseg, const K1Tail* d_tails, uint32_t ntail,
                                      uint32_t nfull, uint32_t B, uint32_t dl, uint32_t seed_word, hipStream_t s) {
    if (nseg + ntail == 0) return hipSuccess;
    // gathered waves for the full-length tails when that adds no wave (the launch fills the chip's 2048 wave
    // slots exactly in the bench's shift case: one more wave would start only when another finished).
    // Option k1_gather = 0: every tail per lane.
    const bool gather_on = tail_gather_on();
    const int* never = never_word();
    uint32_t ngf = 0;
    if (gather_on && never && nfull > 0 && nfull <= ntail && (B % 128) == 0 && (B >> 7) >= 4 &&
        (nfull + 63) / 64 + (ntail - nfull + 63) / 64 == (ntail + 63) / 64)
        ngf = nfull;
    const uint32_t waves = nseg + (ngf + 63) / 64 + (ntail - ngf + 63) / 64;
    // LDS: the shift wave's ring (64 rows of 17 slots); a gathered wave's two 9-slot buffers when there is one
    const size_t lb = ngf > 0 ? 2 * 64 * 9 * sizeof(uint4) : 64 * 17 * sizeof(uint4);
    hipLaunchKernelGGL(block_sums_seg_kernel, dim3(waves), dim3(64), lb, s, d_segs, nseg, d_tails, ntail, B, dl,
                       seed_word, ngf, never);
    return hipGetLastError();
}


constexpr uint32_t kCUs = 256;            // MI355X compute units

// K1 timing (k1_timing_next): the events the next production K1 launch on this thread records with its dispatch.
namespace {
thread_local hipEvent_t t_k1_start = nullptr, t_k1_stop = nullptr;
thread_local bool t_k1_taken = false;
}  // namespace
void k1_timing_next(hipEvent_t start, hipEvent_t stop) {
    t_k1_start = start;
    t_k1_stop = stop;
    t_k1_taken = false;
}
bool k1_timing_taken() { return t_k1_taken; }
// A production K1 launch: with the pending timing events through hipExtLaunchKernelGGL (they are consumed), else
// a plain launch.
template <typename... KArgs, typename... Args>
static void k1_launch(void (*kernel)(KArgs...), dim3 grid, dim3 block, uint32_t lds, hipStream_t s, Args... args) {
    if (t_k1_start) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t_k1_start, t_k1_stop, 0u, static_cast<KArgs>(args)...);
        t_k1_start = t_k1_stop = nullptr;
        t_k1_taken = true;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, static_cast<KArgs>(args)...);
    }
}

// The single-file K1.  variant -1: the production choice -- the pipelined K1 (with its gathered tail) or, at a base
// off a 128-B line, the line-aligned shift kernel; the per-lane kernel for the shapes they do not take.  variant 0
// (kbench's parity reference): the per-lane kernel for every chunk.
#ifndef RSH_KBENCH
static
#endif
hipError_t launch_block_sums_variant(int variant, const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks,
                                     uint32_t dl, uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong,
                                     hipStream_t s, const int* abort_flag, int abort_gen) {
    if (nchunks == 0) return hipSuccess;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(d_data);
    const uint32_t nst = B >> 7;
#ifdef RSH_KBENCH
    if (variant == 1010) {  // the VALU weak-sum form over whole waves (kbench shapes: n = 64 k B, 128-B aligned)
        if ((B % 128) != 0 || nst < 4 || nst > 1024 || n != (int64_t)nchunks * B || nchunks % 64 != 0 || (addr % 128) != 0)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(block_sums_pipe_weakv_kernel, dim3(nchunks / 64), dim3(64), 2 * 64 * 9 * sizeof(uint4), s,
                           d_data, B, dl, seed_word, d_weak, d_strong, abort_flag ? abort_flag : never_word(),
                           abort_flag ? abort_gen : -1);
        return hipGetLastError();
    }
#endif
    // the pipelined and shift kernels poll an abort word (never_word() for launches without one of their own)
    const bool coalesced = variant < 0 && abort_flag && (B % 128) == 0 && nst >= 4 && nst <= 1024;
    // A base that is not 128-B aligned goes to the line-aligned shift kernel when the lines it reads around the
    // data -- a bytes before it, up to 128 - a after the last full wave -- lie in the same allocation (option
    // k1_shift = 0, test: the pipelined kernel at the unaligned base, its path when the lines do not fit).
    if (coalesced && (addr % 128) != 0 && opt(OPT_K1_SHIFT) != 0) {
        hipDeviceptr_t lo = nullptr;
        size_t size = 0;
        const uint32_t a = (uint32_t)(addr % 128);
        if (hipMemGetAddressRange(&lo, &size, reinterpret_cast<hipDeviceptr_t>(const_cast<uint8_t*>(d_data))) ==
                hipSuccess &&
            addr - a >= reinterpret_cast<uintptr_t>(lo)) {
            const int64_t avail = (int64_t)(reinterpret_cast<uintptr_t>(lo) + size - (addr - a));
            const uint32_t nfullc = (uint32_t)std::min<int64_t>(n / B, nchunks);
            const int64_t fit = avail >= 128 ? (avail - 128) / ((int64_t)64 * B) : 0;
            const uint32_t mw = (uint32_t)std::min<int64_t>(nfullc / 64, fit);
            if (mw > 0) {
                uint32_t tail_waves = (nchunks - 64 * mw + 63) / 64;
                // full-length leftovers gathered into coalesced waves when that adds no wave or every wave fits
                // the chip's slots (as block_sums_pipe_tailg_kernel); LDS then for the gathered body's buffers
                const uint32_t tail_full = nfullc - 64 * mw, tail_short = nchunks - nfullc;
                const uint32_t gwaves = (tail_full + 63) / 64 + (tail_short + 63) / 64;
                const bool gather = tail_full > 0 && tail_gather_on() &&
                                    (gwaves == tail_waves || mw + gwaves <= 2 * 4 * kCUs);
                const uint32_t tf = gather ? tail_full : 0u;
                if (gather) tail_waves = gwaves;
                const dim3 grid(mw + tail_waves);
                const size_t lb = gather ? 2 * 64 * 9 * sizeof(uint4) : 64 * 17 * sizeof(uint4);
                switch ((a >> 2) & 3) {
                    case 0:
                        k1_launch(block_sums_shift_kernel<0>, grid, dim3(64), (uint32_t)lb, s, d_data, n, a, B, nchunks,
                                  mw, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, tf);
                        break;
                    case 1:
                        k1_launch(block_sums_shift_kernel<1>, grid, dim3(64), (uint32_t)lb, s, d_data, n, a, B, nchunks,
                                  mw, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, tf);
                        break;
                    case 2:
                        k1_launch(block_sums_shift_kernel<2>, grid, dim3(64), (uint32_t)lb, s, d_data, n, a, B, nchunks,
                                  mw, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, tf);
                        break;
                    default:
                        k1_launch(block_sums_shift_kernel<3>, grid, dim3(64), (uint32_t)lb, s, d_data, n, a, B, nchunks,
                                  mw, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, tf);
                }
                return hipGetLastError();
            }
        }
    }
    // The pipelined K1 also runs at base addresses that are not 16-B aligned (the phase-shifted speculation
    // starts at src + s for any s): its dwordx4 buffer loads then straddle 16-B boundaries, which gfx950
    // serves in its unaligned access mode (bit-exact against the oracle at offsets 0..15,
    // test_k1_unaligned_base).  Option k1_unaligned = 0 (test) sends such bases to the per-lane kernel instead.
    const uint32_t waves = (uint32_t)std::min<int64_t>(n / B, nchunks) / 64;
    if (coalesced && waves > 0 && ((addr % 16) == 0 || opt(OPT_K1_UNALIGNED) != 0)) {
        const uint32_t nfullc = (uint32_t)std::min<int64_t>(n / B, nchunks);  // chunks with L == B
        const size_t wave_lds = 64 * 9 * sizeof(uint4);
        // the pipelined K1 at any wave count (occupancy pinned to 2 waves/SIMD; beyond 2048 waves they run in
        // rounds): measured 3.19 vs 3.96 ms for 16 GiB at B = 64 KiB (4096 waves) against the unpinned
        // instantiation, and ahead of the round-1 coalesced kernel at every size
        const uint32_t tail_waves = (nchunks - 64 * waves + 63) / 64;  // in the same launch
        // the partial last wave's full chunks gathered into a coalesced wave when that adds no wave or every wave
        // still fits the chip's slots (2 per SIMD)
        const uint32_t tail_full = nfullc - 64 * waves, tail_short = nchunks - nfullc;
        const uint32_t gwaves = (tail_full + 63) / 64 + (tail_short + 63) / 64;
        if (tail_full > 0 && tail_gather_on() && (gwaves == tail_waves || waves + gwaves <= 2 * 4 * kCUs)) {
            k1_launch(block_sums_pipe_tailg_kernel, dim3(waves + gwaves), dim3(64), (uint32_t)(2 * wave_lds), s, d_data,
                      B, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, n, nchunks, waves, tail_full);
            return hipGetLastError();
        }
        k1_launch(block_sums_pipe_kernel<false>, dim3(waves + tail_waves), dim3(64), (uint32_t)(2 * wave_lds), s,
                  d_data, B, dl, seed_word, d_weak, d_strong, abort_flag, abort_gen, nullptr, n, nchunks, waves);
        return hipGetLastError();
    }
    // one lane per chunk
    const dim3 block(64);
    const dim3 grid((nchunks + 63) / 64);
    if ((B % 16) == 0 && (addr % 16) == 0) {
        hipLaunchKernelGGL((block_sums_kernel<16, 4, true>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong, 0u);
    } else if ((B % 4) == 0 && (addr % 4) == 0) {
        hipLaunchKernelGGL((block_sums_kernel<4, 2>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word, d_weak,
                           d_strong, 0u);
    } else {
        hipLaunchKernelGGL((block_sums_kernel<0, 4, false>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong, 0u);
    }
    return hipGetLastError();
}

void plan_block_sums_batch(const K1File* files, int32_t nfiles, std::vector<K1Group>* groups,
                           std::vector<K1Lane>* lanes, int* lane_align) {
    groups->clear();
    lanes->clear();
    *lane_align = 16;
    for (int32_t f = 0; f < nfiles; ++f) {
        const K1File& F = files[f];
        if (F.nchunks == 0 || F.B == 0) continue;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(F.data);
        const uint32_t nst = F.B >> 7;
        uint32_t c = 0;
        if ((F.B % 128) == 0 && nst >= 4 && nst <= 1024 && (addr % 16) == 0) {  // the pipelined K1's shape
            const uint32_t nfullc = (uint32_t)std::min<int64_t>(F.n / F.B, F.nchunks);
            for (; c + 64 <= nfullc; c += 64)
                groups->push_back(
                    K1Group{F.data + (size_t)c * F.B, F.weak + c, F.strong + (size_t)c * F.dl, F.B, F.dl, nullptr, f});
        }
        for (; c < F.nchunks; c += 64) {
            lanes->push_back(K1Lane{F.data, F.n, F.weak, F.strong, F.B, F.dl, c, F.nchunks, f});
            const int a = ((F.B % 16) == 0 && (addr % 16) == 0) ? 16 : ((F.B % 4) == 0 && (addr % 4) == 0) ? 4 : 1;
            *lane_align = std::min(*lane_align, a);
        }
    }
}


uint32_t plan_block_sums_files(const K1File* files, int32_t nfiles, std::vector<K1Plan>* plans,
                               std::vector<K1Lane>* lanes, int* lane_align, bool* partial) {
    plans->clear();
    lanes->clear();
    *lane_align = 16;
    bool want_partial = partial && *partial;
    if (partial) *partial = false;
    if (want_partial) {
        // partial groups + one lane per short chunk, or (as without them) one lane wave per file tail: whichever
        // needs fewer rounds of the chip's wave slots (a wave past the last full round waits for a free slot;
        // the lanes run in the same launch, launch_block_sums_batch)
        uint64_t full = 0, w_part = 0, shorts = 0, w_lane = 0;
        for (int32_t f = 0; f < nfiles; ++f) {
            const K1File& F = files[f];
            if (F.nchunks == 0 || F.B == 0) continue;
            const uint32_t nst = F.B >> 7;
            const uintptr_t addr = reinterpret_cast<uintptr_t>(F.data);
            uint32_t nfullc = 0;
            if ((F.B % 128) == 0 && nst >= 4 && nst <= 1024 && (addr % 16) == 0)
                nfullc = (uint32_t)std::min<int64_t>(F.n / F.B, F.nchunks);
            full += nfullc / 64;
            w_part += (nfullc % 64) ? 1 : 0;
            shorts += F.nchunks - nfullc;
            w_lane += (F.nchunks - 64 * (nfullc / 64) + 63) / 64;
        }
        const uint64_t slots = 2ull * 4 * kCUs;
        const uint64_t r_part = (full + w_part + (shorts + 63) / 64 + slots - 1) / slots;
        const uint64_t r_lane = (full + w_lane + slots - 1) / slots;
        want_partial = w_part > 0 && r_part <= r_lane;
    }
    uint32_t g = 0;
    for (int32_t f = 0; f < nfiles; ++f) {  // the same cut as plan_block_sums_batch
        const K1File& F = files[f];
        if (F.nchunks == 0 || F.B == 0) continue;
        const uintptr_t addr = reinterpret_cast<uintptr_t>(F.data);
        const uint32_t nst = F.B >> 7;
        uint32_t c = 0;
        if ((F.B % 128) == 0 && nst >= 4 && nst <= 1024 && (addr % 16) == 0) {
            const uint32_t nfullc = (uint32_t)std::min<int64_t>(F.n / F.B, F.nchunks);
            // the full chunks past the last full wave: a partial group (gathered wave) or lanes
            const uint32_t ng = want_partial ? (nfullc + 63) / 64 : nfullc / 64;
            const uint32_t cov = std::min(nfullc, 64 * ng);
            if (ng > 0) plans->push_back(K1Plan{F.data, F.weak, F.strong, F.B, F.dl, g, ng, nullptr, f, cov});
            if (cov % 64 != 0) *partial = true;
            g += ng;
            c = cov;
        }
        for (; c < F.nchunks; c += 64) {
            lanes->push_back(K1Lane{F.data, F.n, F.weak, F.strong, F.B, F.dl, c, F.nchunks, f});
            const int a = ((F.B % 16) == 0 && (addr % 16) == 0) ? 16 : ((F.B % 4) == 0 && (addr % 4) == 0) ? 4 : 1;
            *lane_align = std::min(*lane_align, a);
        }
    }
    return g;
}

__global__ __launch_bounds__(256) void expand_groups_kernel(const K1Plan* __restrict__ plans, uint32_t nplans,
                                                            uint32_t ngroups, K1Group* __restrict__ groups) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ngroups) return;
    uint32_t lo = 0, hi = nplans;  // the last plan with g0 <= t
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (plans[mid].g0 <= t) lo = mid;
        else hi = mid;
    }
    const K1Plan& P = plans[lo];
    const uint32_t c = 64 * (t - P.g0);
    groups[t] = K1Group{P.data + (size_t)c * P.B, P.weak + c, P.strong + (size_t)c * P.dl, P.B, P.dl, P.abort, P.file,
                        min(64u, P.nfull - c)};
}

hipError_t launch_expand_groups(const K1Plan* d_plans, uint32_t nplans, uint32_t ngroups, K1Group* d_groups,
                                hipStream_t s) {
    if (ngroups == 0 || nplans == 0) return hipSuccess;
    hipLaunchKernelGGL(expand_groups_kernel, dim3((ngroups + 255) / 256), dim3(256), 0, s, d_plans, nplans, ngroups,
                       d_groups);
    return hipGetLastError();
}

// A word no launch ever writes: non-abortable K1 launches run the abortable instantiation polling it with
// generation -1 (never stored).  Measured on the MI355X pool (round 2, kbench 16 GiB at B = 128 KiB, same
// process, same buffer): the plain instantiation 4.07-4.57 ms, the abortable one 2.99-3.10 ms (the plain one
// with only the abortable loop's lgkmcnt(0) drain: 4.38 ms); round 1's boxes ran both at ~3.0 ms.  The word
// must be uncached device memory like the contexts' abort words: polling a __device__ global instead (L2,
// one line for every wave) made the launch 27.9 ms.
static const int* never_word() {
    static int* ptr[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (!ptr[dev]) {  // one 256-B uncached word per device for the process's lifetime
        int* p = nullptr;
        if (hipExtMallocWithFlags(reinterpret_cast<void**>(&p), 256, hipDeviceMallocUncached) != hipSuccess) return nullptr;
        if (hipMemset(p, 0, 256) != hipSuccess) return nullptr;
        ptr[dev] = p;
    }
    return ptr[dev];
}

// The batched K1 with its leftovers in the same launch: groups some of which are a file's partial last wave
// (K1Group::count < 64: the gathered-wave path, one 64-bit pointer per 8-chunk row, lanes past the count store
// nothing), then the lane waves (short chunks and odd shapes, one chunk per lane), instead of the per-lane
// kernel queued behind the groups (a wave of it takes one chunk's serial time: ~2 ms at B = 128 KiB).
// Register budget 256 as block_sums_pipe_tailg_kernel.
template <int ALIGN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(256))) void block_sums_pipe_multi_g_kernel(
    const K1Group* __restrict__ groups, uint32_t ngroups, const K1Lane* __restrict__ lanes, uint32_t seed,
    const int* abort_flag, int abort_gen) {
    if (blockIdx.x >= ngroups) {  // the lane waves (short chunks, odd shapes) in the same launch
        const K1Lane e = lanes[blockIdx.x - ngroups];
        const uint32_t c = e.c_first + threadIdx.x;
        if (c < e.nchunks)
            lane_chunk_sums<ALIGN == 1 ? 0 : ALIGN, ALIGN == 16 ? 4 : ALIGN == 4 ? 2 : 4, ALIGN != 1>(
                e.data, e.n, e.B, c, e.dl, seed, e.weak, e.strong);
        return;
    }
    const K1Group g = groups[blockIdx.x];
    if (g.count < 64) {
        block_sums_pipe_body<false, true>(g.data, g.B, g.dl, seed, g.weak, g.strong,
                                                           g.abort ? g.abort : abort_flag, abort_gen, nullptr, 0, 0,
                                                           0xFFFFFFFFu, nullptr, g.count);
        return;
    }
    block_sums_pipe_body<true>(nullptr, 0u, 0u, seed, nullptr, nullptr, abort_flag, abort_gen, groups);
}

hipError_t launch_block_sums_batch(const K1Group* d_groups, uint32_t ngroups, const K1Lane* d_lanes, uint32_t nlanes,
                                   int lane_align, uint32_t seed_word, hipStream_t s, const int* abort_flag,
                                   int abort_gen, bool partial) {
    const size_t lb = 2 * 64 * 9 * sizeof(uint4);
    if (!abort_flag && (abort_flag = never_word()) != nullptr) abort_gen = -1;  // see never_word
    if (!abort_flag) return hipErrorOutOfMemory;  // never_word() failed: no uncached word for the pinned K1
    // partial groups, or lanes beside groups: one launch (option k1_gather = 0: the lanes as a second launch)
    if (partial || (tail_gather_on() && nlanes > 0 && ngroups > 0)) {
        const dim3 grid(ngroups + nlanes);
        if (lane_align == 16)
            hipLaunchKernelGGL((block_sums_pipe_multi_g_kernel<16>), grid, dim3(64), lb, s, d_groups, ngroups, d_lanes,
                               seed_word, abort_flag, abort_gen);
        else if (lane_align == 4)
            hipLaunchKernelGGL((block_sums_pipe_multi_g_kernel<4>), grid, dim3(64), lb, s, d_groups, ngroups, d_lanes,
                               seed_word, abort_flag, abort_gen);
        else
            hipLaunchKernelGGL((block_sums_pipe_multi_g_kernel<1>), grid, dim3(64), lb, s, d_groups, ngroups, d_lanes,
                               seed_word, abort_flag, abort_gen);
        return hipGetLastError();
    }
    if (ngroups > 0)
        hipLaunchKernelGGL((block_sums_pipe_kernel<true>), dim3(ngroups), dim3(64), lb, s, nullptr, 0u, 0u, seed_word,
                           nullptr, nullptr, abort_flag, abort_gen, d_groups);
    if (nlanes > 0) {
        if (lane_align == 16)
            hipLaunchKernelGGL((block_sums_lane_batch_kernel<16>), dim3(nlanes), dim3(64), 0, s, d_lanes, seed_word);
        else if (lane_align == 4)
            hipLaunchKernelGGL((block_sums_lane_batch_kernel<4>), dim3(nlanes), dim3(64), 0, s, d_lanes, seed_word);
        else
            hipLaunchKernelGGL((block_sums_lane_batch_kernel<1>), dim3(nlanes), dim3(64), 0, s, d_lanes, seed_word);
    }
    return hipGetLastError();
}

hipError_t launch_block_sums(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks, uint32_t dl,
                             uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong, hipStream_t s,
                             const int* abort_flag, int abort_gen) {
    if (!abort_flag && (abort_flag = never_word()) != nullptr) abort_gen = -1;
    return launch_block_sums_variant(-1, d_data, n, B, nchunks, dl, seed_word, d_weak, d_strong, s, abort_flag,
                                     abort_gen);
}

// ------------------------------------------------------------------------------------------------
// Chain flags (Sender fast path): the aligned source window k would be matched against chunk k.
// ------------------------------------------------------------------------------------------------
__global__ void chain_flags_kernel(const int32_t* __restrict__ wsrc, const uint8_t* __restrict__ ssrc,
                                   const int32_t* __restrict__ wbas, const uint8_t* __restrict__ sbas,
                                   uint32_t count, uint32_t dl, uint8_t* __restrict__ flags) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    bool eq = wsrc[k] == wbas[k];
    for (uint32_t j = 0; j < dl; ++j) eq &= ssrc[(size_t)k * dl + j] == sbas[(size_t)k * dl + j];
    flags[k] = eq ? 1 : 0;
}

hipError_t launch_chain_flags(const int32_t* d_wsrc, const uint8_t* d_ssrc, const int32_t* d_wbas,
                              const uint8_t* d_sbas, uint32_t count, uint32_t dl, uint8_t* d_flags,
                              hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_flags_kernel, dim3((count + 255) / 256), dim3(256), 0, s, d_wsrc, d_ssrc, d_wbas,
                       d_sbas, count, dl, d_flags);
    return hipGetLastError();
}

// A kernel that does nothing: its first launch makes the runtime load this file's code object (the K1 kernels) --
// 0.6-1.8 ms on a fresh context, which rsh_ctx_create pays instead of the first call (launch_warm).
__global__ void warm_k1_kernel() {}
hipError_t launch_warm_k1(hipStream_t s) {
    if (!never_word()) return hipErrorOutOfMemory;  // (allocated once per device; the Generator's K1 polls it)
    hipLaunchKernelGGL(warm_k1_kernel, dim3(1), dim3(64), 0, s);
    return hipGetLastError();
}

}  // namespace rsh
