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

__device__ __forceinline__ int32_t sbyte(uint8_t v) { return (int32_t)(int8_t)v; }

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

// ------------------------------------------------------------------------------------------------
// K1 (coalesced): one wave owns 64 consecutive full-length chunks (L = B, B % 128 == 0).  A stage is
// the next 128 B of every chunk: 8 global_load_dwordx4 per lane, each instruction reading 8 whole
// 128-B lines (8 lanes per line) instead of 64 scattered 16-B pieces; the wave transposes the stage
// through LDS (row = 8 data slots + 1 pad slot, so the 16-lane ds_read_b128 groups and the 8-lane
// ds_write_b128 groups are both bank-conflict free) and each lane then runs its chunk's MD5 over the
// two 64-B blocks.  D stages stay in flight in registers.
// ------------------------------------------------------------------------------------------------
// Wave-local ordering of the stage transpose: LDS operations of one wave execute in order, so only
// the compiler has to be kept from moving the lane-crossing ds_read above the ds_write (or the next
// stage's ds_write above this stage's ds_read).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MODE (diagnostics only, never in the production launch): 0 = real, 1 = compute only (no global
// loads; stage data synthesised in registers), 2 = loads only (no MD5/weak; words xor-folded).
typedef int v4i32 __attribute__((ext_vector_type(4)));

// Weak sums on the matrix pipe (MFMAW): per stage, for each group g of 16 chunks and K-half h,
// C_g += W_h x X_{g,h} with v_mfma_i32_16x16x64_i8, where X holds 64 signed bytes of 16 chunks
// (columns) and W_h has row 0 = ones and row 1 = the byte's index in the 128-B stage (<= 127, int8).
// Row 0 of C accumulates s1; row 1 accumulates the in-stage-index-weighted sums; R_g += row 0 after
// every stage gives sum_s P_s, so u = sum_i i x_i = 128 (nst * P_last - R) + row1.  Column j of group g
// is chunk 16g + kPi[j] and K-slice s reads piece 4h + kSigma[s]: with the 9-slot LDS rows every
// 16-lane ds_read_b128 group then hits 16 distinct bank quads (checked exhaustively).
__device__ __forceinline__ int mfma_pi(int j) { return (int)((0xECA8FDB975316420ull >> (4 * j)) & 15); }
__device__ __forceinline__ int mfma_pi_inv(int c) { return (int)((0xBFAE9D8C73625140ull >> (4 * c)) & 15); }
__device__ __forceinline__ int mfma_sigma(int s) { return (0x1302 >> (4 * s)) & 15; }

// ABORT (the Sender's speculation only): every 16 stages the wave reads *abort_flag (uncached device
// memory, set by a stream write-value packet) with a cache-bypassing scalar load and exits when it
// equals abort_gen -- the resolver finished without needing this launch's results.  The read waits
// for itself only (the LDS traffic of the iteration is consumed by then; vector loads are untouched).
__device__ __forceinline__ int poll_abort(const int* flag) {
    int v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(flag));
    return v;
}

template <int D, bool NT, int WAVES = 1, int MODE = 0, bool FUSED = false, bool MFMAW = false, bool STEADY = true,
          bool ABORT = false, int MD5F = 2, bool PIN = false>
__global__ __launch_bounds__(64 * WAVES) void block_sums_coalesced_kernel(const uint8_t* __restrict__ data, uint32_t B,
                                                                  uint32_t dl, uint32_t seed,
                                                                  int32_t* __restrict__ weak_out,
                                                                  uint8_t* __restrict__ strong_out,
                                                                  const int* abort_flag = nullptr,
                                                                  int abort_gen = 0) {
    constexpr int ROW = 9;
    // MODE (diagnostics): 0 production, 1 synthetic stage data (no loads), 2 no MD5, 3 = 1 without the weak-sum
    // MFMAs, 4 = 3 without the LDS transpose (MD5 on the raw register words)
    constexpr bool SYN = MODE == 1 || MODE == 3 || MODE == 4;
    // PIN: claim VGPRs up to v183 so that at most 2 waves fit a SIMD (512 / 184).  The MFMAW body needs 156,
    // which admits 3; a launch with exactly 2 waves per SIMD of work (16 GiB at B = 128 KiB) then may stack
    // 3 on some SIMDs and 1 on others when it starts while another kernel drains (5.1 ms instead of 3.2).
    if constexpr (PIN) asm volatile("; occupancy pin" ::: "v183");
    extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // sized at launch (occupancy control)
    const int l = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    uint4* lds = lds_all + wv * 64 * ROW;
    const uint32_t c0 = (blockIdx.x * WAVES + wv) * 64u;
    const uint32_t nst = B >> 7;
    const uint8_t* lp = data + ((size_t)c0 + (size_t)(l >> 3)) * B + 16 * (l & 7);
    const size_t jstride = (size_t)8 * B;
    const int wr0 = (l >> 3) * ROW + (l & 7);
    const int rd0 = l * ROW;

    uint4 q[D][8];
    uint32_t fold = 0;
    // MFMAW state: weights (row 0 ones, row 1 in-stage byte index), accumulators, running R
    v4i32 wA[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    v4i32 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    int32_t Racc[4] = {0, 0, 0, 0};
    int rdB = 0;
    if constexpr (MFMAW) {
        const int row = l & 15, ks = l >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t word = 0;
                if (row == 0) word = 0x01010101u;
                else if (row == 1)
#pragma unroll
                    for (int b = 0; b < 4; ++b) word |= (uint32_t)(16 * (4 * h + mfma_sigma(ks)) + 4 * w + b) << (8 * b);
                wA[h][w] = (int)word;
            }
        rdB = mfma_pi(l & 15) * ROW + mfma_sigma(ks);
    }
    // host guarantees nst >= 2 * D: the prologue is unconditional (exact vmcnt bookkeeping)
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (SYN) q[d][j] = make_uint4(l + d, j, c0, 7);
            else q[d][j] = ld16<NT>(lp + 128 * (size_t)d + j * jstride);
        }
    }
    Md5State st = md5_init();
    int32_t s1 = 0, u = 0;
    // One stage: registers -> LDS (transpose), refill the registers PF stages ahead, weak sums on the
    // matrix pipe (MFMAW) and the two MD5 blocks.  Inlined with a compile-time slot d.
    auto stage = [&](auto dc, uint32_t si, bool refill) __attribute__((always_inline)) {
        constexpr int d = decltype(dc)::value;
        uint4 qs[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            qs[j] = q[d][j];
            if constexpr (MODE != 4) lds[wr0 + j * 8 * ROW] = q[d][j];
        }
        if (refill) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if constexpr (SYN) q[d][j] = make_uint4(q[d][j].y + si, q[d][j].x, q[d][j].w ^ si, q[d][j].z);
                else q[d][j] = ld16<NT>(lp + 128 * (size_t)(si + D) + j * jstride);
            }
        }
        if constexpr (MODE == 4) {
        } else if constexpr (WAVES == 1) __syncthreads();
        else wave_lds_sync();
        if constexpr (MFMAW && MODE != 3 && MODE != 4) {
#pragma unroll
            for (int g = 0; g < 4; ++g) Racc[g] += acc[g][0];  // R += P_{s-1}
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const uint4 bv = lds[16 * ROW * g + rdB + 4 * h];
                    const v4i32 b4 = {(int)bv.x, (int)bv.y, (int)bv.z, (int)bv.w};
                    acc[g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wA[h], b4, acc[g], 0, 0, 0);
                }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint4 r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = MODE == 4 ? qs[4 * h + k] : lds[rd0 + 4 * h + k];
            uint32_t m[16];
            unpack(r, m);
            if constexpr (MODE == 2) {
#pragma unroll
                for (int k = 0; k < 16; ++k) fold ^= m[k];
            } else if constexpr (MFMAW) {
                if constexpr (MD5F == 8) md5_compress_rot16n(st, m);
#ifdef RSH_KBENCH
    else if constexpr (MD5F == 10) md5_compress_k3s_8(st, m);   // A/B: a + m + K in one v_add3_u32, K from an SGPR
    else if constexpr (MD5F == 11) md5_compress_k3s_16(st, m);
    else if constexpr (MD5F == 12) md5_compress_k3s_16_nonop(st, m);
    else if constexpr (MD5F == 13) md5_compress_k3s_16_nop2(st, m);
#endif
                else if constexpr (MD5F == 7) md5_compress_rot4n(st, m);
                else if constexpr (MD5F == 6) md5_compress_rot16(st, m);
                else if constexpr (MD5F == 5) md5_compress_rot4(st, m);
                else if constexpr (MD5F == 4) md5_compress_asm16(st, m);
                else if constexpr (MD5F == 3) md5_compress_asm4(st, m);
                else if constexpr (MD5F == 2) md5_compress_asm(st, m);
                else if constexpr (MD5F == 1) md5_compress_lit(st, m);
                else md5_compress(st, m);
            } else if constexpr (FUSED && MD5F == 1) {
                int32_t wa, wb;
                md5_compress_lit_weak(st, m, wa, wb);
                s1 += wa;
                u += (int32_t)((128 * si + 64 * h) * (uint32_t)wa) + wb;
            } else if constexpr (FUSED) {
                md5_weak_block(st, m, s1, u, 128 * si + 64 * h);
            } else {
                weak_block(m, s1, u, 128 * si + 64 * h);
                md5_compress(st, m);
            }
        }
        if constexpr (MODE == 4) {
        } else if constexpr (WAVES == 1) __syncthreads();
        else wave_lds_sync();
    };
    uint32_t s = 0;
    if constexpr (!STEADY) {  // A/B reference: conditional refills in one loop
        for (; s < nst; s += D) {
            if (s < nst) stage(std::integral_constant<int, 0>{}, s, s + D < nst);
            if constexpr (D > 1) if (s + 1 < nst) stage(std::integral_constant<int, 1>{}, s + 1, s + 1 + D < nst);
            if constexpr (D > 2) if (s + 2 < nst) stage(std::integral_constant<int, 2>{}, s + 2, s + 2 + D < nst);
        }
    }
    // steady state: branch-free, every slot refilled, so the compiler's vmcnt bookkeeping stays exact
    // (with conditional refills it waits for every outstanding load at each stage: prefetch depth 1)
    for (; s + 2 * D <= nst; s += D) {
        stage(std::integral_constant<int, 0>{}, s, true);
        if constexpr (D > 1) stage(std::integral_constant<int, 1>{}, s + 1, true);
        if constexpr (D > 2) stage(std::integral_constant<int, 2>{}, s + 2, true);
        if constexpr (D > 3) stage(std::integral_constant<int, 3>{}, s + 3, true);
        if constexpr (ABORT) {
            if ((s & 15) == 0 && poll_abort(abort_flag) == abort_gen) return;
        }
    }
    for (; s < nst; s += D) {  // drain (fewer than 2 * D stages left)
        if (s < nst) stage(std::integral_constant<int, 0>{}, s, s + D < nst);
        if constexpr (D > 1) if (s + 1 < nst) stage(std::integral_constant<int, 1>{}, s + 1, s + 1 + D < nst);
        if constexpr (D > 2) if (s + 2 < nst) stage(std::integral_constant<int, 2>{}, s + 2, s + 2 + D < nst);
        if constexpr (D > 3) if (s + 3 < nst) stage(std::integral_constant<int, 3>{}, s + 3, s + 3 + D < nst);
    }
    // final block: seed || 0x80 || zero pad || bit length of (B + 4) bytes
    {
        const uint64_t bits = ((uint64_t)B + 4) * 8;
        uint32_t m[16] = {seed, 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, (uint32_t)bits, (uint32_t)(bits >> 32)};
        md5_compress(st, m);
    }
    if constexpr (MFMAW) {
        // lanes 0..15 of group g hold (P_last, row1, R) for chunk 16g + pi(lane); move them to lane c
        int32_t s1g[4], ug[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            Racc[g] += acc[g][0];
            s1g[g] = acc[g][0];
            ug[g] = (int32_t)(128u * (nst * (uint32_t)acc[g][0] - (uint32_t)Racc[g])) + acc[g][1];
        }
        const int src = mfma_pi_inv(l & 15);
        int32_t t1[4], tu[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            t1[g] = __shfl(s1g[g], src, 64);
            tu[g] = __shfl(ug[g], src, 64);
        }
        const int gs = l >> 4;
        s1 = gs == 0 ? t1[0] : gs == 1 ? t1[1] : gs == 2 ? t1[2] : t1[3];
        u = gs == 0 ? tu[0] : gs == 1 ? tu[1] : gs == 2 ? tu[2] : tu[3];
    }
    const uint32_t c = c0 + l;
    if constexpr (MODE == 2) st.a ^= fold;
    const int32_t s2 = (int32_t)(B * (uint32_t)s1 - (uint32_t)u);
    weak_out[c] = (int32_t)(((uint32_t)s1 & 0xFFFFu) | ((uint32_t)s2 << 16));
    store_digest(strong_out + (size_t)c * dl, st, dl);
}

// ------------------------------------------------------------------------------------------------
// K1, software-pipelined (production).  Same data path as block_sums_coalesced_kernel (coalesced
// 128-B-line loads, LDS transpose with 9-slot rows, weak sums on the matrix pipe, one lane = one chunk),
// but no LDS round trip ever sits on a wave's critical path: stage s+1 is written to the second LDS
// buffer at the top of stage s, its message words and MFMA operands are read back into registers
// between the two MD5 blocks of stage s, so they have landed long before stage s+1 starts.  The weak-sum
// MFMAs of stage s sit between its MD5 blocks too.  Two stages of loads stay in flight (slots q[0..1]).
// LDS operations of one wave execute in order, so a compiler-only barrier orders the write and the
// reads of a buffer; no s_waitcnt lgkmcnt(0) / s_barrier per stage.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// MD5F == 9 (kbench A/B): the K constants in VGPRs, a + m + K as one v_add3_u32 (gfx950 VOP3 has no literal)
__device__ __forceinline__ void md5_k3_init(uint32_t (&kv)[64]) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(__gfx950__)
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        kv[i] = RSH_MD5_KTAB[i];
        asm volatile("" : "+v"(kv[i]));
    }
#endif
}
__device__ __forceinline__ void md5_k3_block(Md5State& st, const uint32_t (&m)[16], const uint32_t (&kv)[64]) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(__gfx950__)
    md5_compress_k3_8(st, m, kv);
#endif
}
template <int MD5F>
__device__ __forceinline__ void md5_stream_block(Md5State& st, const uint32_t (&m)[16]) {
    if constexpr (MD5F == 8) md5_compress_rot16n(st, m);
#ifdef RSH_KBENCH
    else if constexpr (MD5F == 10) md5_compress_k3s_8(st, m);   // A/B: a + m + K in one v_add3_u32, K from an SGPR
    else if constexpr (MD5F == 11) md5_compress_k3s_16(st, m);
    else if constexpr (MD5F == 12) md5_compress_k3s_16_nonop(st, m);
    else if constexpr (MD5F == 13) md5_compress_k3s_16_nop2(st, m);
#endif
    else if constexpr (MD5F == 7) md5_compress_rot4n(st, m);
    else if constexpr (MD5F == 1) md5_compress_lit(st, m);
    else md5_compress(st, m);
}

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
// MODE != 0 (A/B and diagnostic forms: synthetic stage data, per-iteration drains or sleeps) exists in the kbench
// build only (RSH_KBENCH); the product library instantiates MODE 0.
// WEAKW (production since round 4): the weak sums from the MD5 message words already in registers instead of a second read of
// the stage from LDS in the MFMA operand layout: per 64-B block, four v_mfma_i32_16x16x64_i8 with B = the lane's
// own 16-byte quarter w of its block and A = rows that select one lane group each (row m reads lane group m & 3:
// type m >> 2 = 0 ones, 1 the byte's offset 16 w + i in the block), all into one accumulator -- chunk n + 16 q's
// block sum lands in lane n (element q), its weighted sum in lane n + 16.  Saves the 8 ds_read_b128 per stage: the
// same cycles at a higher clock, 2.5 % less time (kbench 66 vs 67, profiles/r4/r4e_kbench_weakw_k3s*).
template <int MD5F, bool ABORT, bool PIN, int MODE = 0, bool MULTI = false, bool GATHER = false, bool WEAKW = true>
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
#ifndef RSH_KBENCH
    static_assert(MODE == 0 && MD5F == 8 && WEAKW, "the product library runs the production K1 only");
#endif
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
    if constexpr (PIN) asm volatile("; occupancy pin" ::: "v175");
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
        if constexpr (ABORT) {
            if (g.abort) abort_flag = g.abort;  // per-file cancellation (batched Sender speculation)
        }
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

    v4i32 wA[2];
    v4i32 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    int32_t Racc[4] = {0, 0, 0, 0};
    {
        const int row = l & 15, ks = l >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t word = 0;
                if (row == 0) word = 0x01010101u;
                else if (row == 1)
#pragma unroll
                    for (int b = 0; b < 4; ++b) word |= (uint32_t)(16 * (4 * h + mfma_sigma(ks)) + 4 * w + b) << (8 * b);
                wA[h][w] = (int)word;
            }
    }
    const int rdB = mfma_pi(l & 15) * ROW + mfma_sigma(l >> 4);
    [[maybe_unused]] v4i32 wW[4];  // WEAKW: the A operand for block quarter w
    [[maybe_unused]] v4i32 accW = {0, 0, 0, 0}, RW = {0, 0, 0, 0};
    if constexpr (WEAKW) {
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
    uint4 Bv[8];    // MFMA operands of the current stage
    // Buffer loads: the wave's 64 chunks (64 * B <= 8 MiB) behind one descriptor, a 32-bit lane offset and
    // a scalar offset per 8-chunk row j -- one VGPR of addressing instead of eight 64-bit pointers.
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(gdata), 0, (int)(64 * B), 0x00020000);
    const uint32_t lane_off = (uint32_t)(l >> 3) * B + 16u * (uint32_t)(l & 7);
    auto load = [&](uint4 (&dst)[8], uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#ifdef RSH_KBENCH
            if constexpr (MODE == 1) {  // diagnostics: synthetic stage data, no global loads
                dst[j] = make_uint4(l + stg, j, c0, 7);
                continue;
            }
#endif
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
    auto get_mfma = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int g = 0; g < 4; ++g) Bv[4 * h + g] = lds_all[buf * BUF + 16 * ROW * g + rdB + 4 * h];
    };
    Md5State st = md5_init();
    // MD5F == 9 (kbench A/B): a + m + K as one v_add3_u32 per step, the 64 K constants held in VGPRs
    [[maybe_unused]] uint32_t kv[64];
    if constexpr (MD5F == 9) md5_k3_init(kv);
    auto md5_block = [&](const uint4 (&w)[4]) __attribute__((always_inline)) {
        uint32_t m[16];
        unpack(w, m);
        if constexpr (MD5F == 9) md5_k3_block(st, m, kv);
        else md5_stream_block<MD5F>(st, m);
    };
    auto weak_words = [&](const uint4 (&w)[4]) __attribute__((always_inline)) {  // WEAKW: one 64-B block
#pragma unroll
        for (int e = 0; e < 4; ++e) RW[e] += accW[e];  // R += P_{b-1}
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const v4i32 b4 = {(int)w[k].x, (int)w[k].y, (int)w[k].z, (int)w[k].w};
            accW = __builtin_amdgcn_mfma_i32_16x16x64_i8(wW[k], b4, accW, 0, 0, 0);
        }
    };
    auto weak_mfma = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) Racc[g] += acc[g][0];  // R += P_{s-1}
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint4 bv = Bv[4 * h + g];
                const v4i32 b4 = {(int)bv.x, (int)bv.y, (int)bv.z, (int)bv.w};
                acc[g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wA[h], b4, acc[g], 0, 0, 0);
            }
    };
    // One stage with compile-time parity P: LDS buffer P holds it, q[P ^ 1] the next stage's data.
    // Block-1 words and MFMA operands are read at the top (they land during block 0); the next stage's
    // block-0 words are read between the blocks (they land during block 1).
    auto stage = [&](auto pc, uint32_t si, bool has_next, bool refill) __attribute__((always_inline)) {
        constexpr int P = decltype(pc)::value;
        if (has_next) {
            put(q[P ^ 1], P ^ 1);
            if (refill) load(q[P ^ 1], si + 3);
        }
        get_words(Wb, P, 1);
        if constexpr (!WEAKW) get_mfma(P);
        md5_block(Wa);
        if constexpr (WEAKW) weak_words(Wa);
        else weak_mfma();
        compiler_fence();
        if (has_next) get_words(Wa, P ^ 1, 0);
        md5_block(Wb);
        if constexpr (WEAKW) weak_words(Wb);
        compiler_fence();
    };

    load(q[0], 0);
    load(q[1], 1);
    if constexpr (ABORT && MULTI) {  // a group whose file was resolved before the wave started does nothing
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
    // ABORT: one scalar load (glc: from L2, not the scalar cache) of the abort word per 2 stages, issued at
    // the top of the iteration and compared at the bottom, so its latency hides behind the two stages.
    // The compiler does not see the load; its own lgkmcnt(N) waits for LDS stay safe with one extra
    // operation in flight (they only get stricter).
    [[maybe_unused]] int flag = 0;
    for (; s + 5 <= nst && (!ABORT || flag != abort_gen); s += 2) {
        if constexpr (ABORT) asm volatile("s_load_dword %0, %1, 0x0 glc" : "=s"(flag) : "s"(abort_flag));
        stage(std::integral_constant<int, 0>{}, s, true, true);
        stage(std::integral_constant<int, 1>{}, s + 1, true, true);
        if constexpr (ABORT) asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(flag));
#ifdef RSH_KBENCH
        else if constexpr (MODE == 5) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // A/B: the drain alone
        else if constexpr (MODE == 6) asm volatile("s_sleep 1" ::: "memory");            // A/B: a short sleep
        else if constexpr (MODE == 7) asm volatile("s_sleep 4" ::: "memory");
#endif
    }
    if constexpr (ABORT) {
        if (flag == abort_gen) return;
    }
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
    if constexpr (WEAKW) {
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
    } else {
        int32_t s1g[4], ug[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            Racc[g] += acc[g][0];
            s1g[g] = acc[g][0];
            ug[g] = (int32_t)(128u * (nst * (uint32_t)acc[g][0] - (uint32_t)Racc[g])) + acc[g][1];
        }
        const int src = mfma_pi_inv(l & 15);
        int32_t t1[4], tu[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            t1[g] = __shfl(s1g[g], src, 64);
            tu[g] = __shfl(ug[g], src, 64);
        }
        const int gs = l >> 4;
        s1 = gs == 0 ? t1[0] : gs == 1 ? t1[1] : gs == 2 ? t1[2] : t1[3];
        u = gs == 0 ? tu[0] : gs == 1 ? tu[1] : gs == 2 ? tu[2] : tu[3];
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

template <int MD5F, bool ABORT, bool PIN, int MODE = 0, bool MULTI = false>
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_kernel(const uint8_t* __restrict__ data, uint32_t B, uint32_t dl,
                                                             uint32_t seed, int32_t* __restrict__ weak_out,
                                                             uint8_t* __restrict__ strong_out,
                                                             const int* abort_flag = nullptr, int abort_gen = 0,
                                                             const K1Group* __restrict__ groups = nullptr,
                                                             int64_t n = 0, uint32_t nchunks = 0,
                                                             uint32_t main_waves = 0xFFFFFFFFu) {
    block_sums_pipe_body<MD5F, ABORT, PIN, MODE, MULTI>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen,
                                                        groups, n, nchunks, main_waves);
}
// The production K1 with the partial last wave's full-length chunks as a gathered coalesced wave (the tail
// waves past main_waves: ceil(tail_full / 64) gathered ones, then the short last chunk, if any, per lane).  A
// per-lane wave runs ~20% slower than a coalesced one and, when every wave runs in the first round, sets the
// launch's end.  Used only for launches with such a tail: the exact-multiple launches keep
// block_sums_pipe_kernel.  Its register budget is 256 (2 waves/SIMD): under K1_PIPE_ATTR the two bodies spill.
template <bool ABORT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(256))) void block_sums_pipe_tailg_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen, int64_t n, uint32_t nchunks,
    uint32_t main_waves, uint32_t tail_full) {
    if (blockIdx.x >= main_waves) {
        const uint32_t tw = blockIdx.x - main_waves, ngw = (tail_full + 63u) / 64u;
        if (tw < ngw) {
            const uint32_t first = main_waves * 64u + 64u * tw;
            block_sums_pipe_body<8, ABORT, true, 0, false, true>(
                data + (size_t)first * B, B, dl, seed, weak_out + first, strong_out + (size_t)first * dl, abort_flag,
                abort_gen, nullptr, 0, 0, 0xFFFFFFFFu, nullptr, min(64u, tail_full - 64u * tw));
            return;
        }
        const uint32_t c = main_waves * 64u + tail_full + (tw - ngw) * 64u + threadIdx.x;
        if (c < nchunks) lane_chunk_sums<16, RSH_K1_TAIL_PF, false>(data, n, B, c, dl, seed, weak_out, strong_out);
        return;
    }
    block_sums_pipe_body<8, ABORT, true, 0, false>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen,
                                                   nullptr, n, nchunks, main_waves);
}
bool tail_gather_on() { return opt(OPT_K1_GATHER) != 0; }  // 0: leftover chunks one per lane (options.h)

// Diagnostic (rsh_debug_k1_clock, MI355X_MICROARCH.md "DVFS give-back" item 6): the Generator's production K1 body
// with each wave's shader-clock (s_memtime) and 100 MHz (s_memrealtime) ticks stamped around it and summed over the
// launch; their quotient x 100 MHz is the clock the chip held under this load.  Only this instantiation stamps: the
// production kernels never execute a stamp.  Whole coalesced waves only (n = 64 k B, B % 128 == 0).
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_clock_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen, int64_t n, uint32_t nchunks,
    unsigned long long* __restrict__ clk) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    block_sums_pipe_body<8, true, true, 0, false>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen,
                                                   nullptr, n, nchunks, 0xFFFFFFFFu);
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
#ifdef RSH_KBENCH
// kbench A/B (variant 67): round 3's production form, the weak-sum MFMA operands read from LDS (WEAKW = false)
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_ldsw_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen) {
    block_sums_pipe_body<8, true, true, 0, false, false, false>(data, B, dl, seed, weak_out, strong_out, abort_flag,
                                                                abort_gen, nullptr, 0, 0, 0xFFFFFFFFu);
}
// kbench A/B (variant 66): the weak sums from the MD5 words in registers (WEAKW; the production form since round 4)
__global__ __launch_bounds__(64) K1_PIPE_ATTR void block_sums_pipe_weakw_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen) {
    block_sums_pipe_body<8, true, true, 0, false, false, true>(data, B, dl, seed, weak_out, strong_out, abort_flag,
                                                               abort_gen, nullptr, 0, 0, 0xFFFFFFFFu);
}
// kbench A/B (variant 61): MD5F == 9 holds the 64 K constants in VGPRs (176 + 64 registers, still 2 waves/SIMD)
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(256))) void block_sums_pipe_k3_kernel(
    const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed, int32_t* __restrict__ weak_out,
    uint8_t* __restrict__ strong_out, const int* abort_flag, int abort_gen) {
    block_sums_pipe_body<9, true, true, 0, false>(data, B, dl, seed, weak_out, strong_out, abort_flag, abort_gen,
                                                  nullptr, 0, 0, 0xFFFFFFFFu);
}
#endif


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
//  * Weak sums: the MFMAs sum whole lines 0..nst in the aligned kernel's operand layout; line 0's bytes before
//    the chunk (a) and line nst's bytes after it (128 - a) are subtracted per lane (v_dot4 over its own row).
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
    const uint32_t c0 = 0;
    const uint32_t nst = B >> 7;  // host guarantees 4 <= nst <= 1024
    const uint32_t Q = a >> 4, r = a & 3;
    const int wr0 = (l >> 3) * ROW + (l & 7);
    const int row = l * ROW;

    v4i32 wA[2];
    v4i32 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    int32_t Racc[4] = {0, 0, 0, 0};
    {
        const int rw = l & 15, ks = l >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t word = 0;
                if (rw == 0) word = 0x01010101u;
                else if (rw == 1)
#pragma unroll
                    for (int b = 0; b < 4; ++b) word |= (uint32_t)(16 * (4 * h + mfma_sigma(ks)) + 4 * w + b) << (8 * b);
                wA[h][w] = (int)word;
            }
    }
    const int rdB = mfma_pi(l & 15) * ROW + mfma_sigma(l >> 4);

    uint4 q[2][8];  // line u + 1 and u + 2 in flight while step u computes
    uint4 Wa[5];    // block 0 of the next MD5 stage
    uint4 Wb[5];    // block 1 of the current MD5 stage
    uint4 Bv[8];    // MFMA operands of the current line
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
    auto get_mfma = [&](int half) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int g = 0; g < 4; ++g) Bv[4 * h + g] = lds_all[16 * ROW * g + rdB + 8 * half + 4 * h];
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
        md5_stream_block<8>(st, m);
    };
    auto weak_mfma = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) Racc[g] += acc[g][0];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint4 bv = Bv[4 * h + g];
                const v4i32 b4 = {(int)bv.x, (int)bv.y, (int)bv.z, (int)bv.w};
                acc[g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wA[h], b4, acc[g], 0, 0, 0);
            }
    };
    // signed-byte sums of the lane's own row, line in `half`, over the bytes j with (j < a) == BEFORE
    auto edge_sums = [&](int half, bool before, int32_t& s, int32_t& u) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = lds_all[row + 8 * half + k];
            const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j0 = 16 * k + 4 * e;
                const int nb = (int)a - j0;  // bytes of this dword before the chunk
                const uint32_t lo = nb <= 0 ? 0u : nb >= 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1u;
                const uint32_t x = dw[e] & (before ? lo : ~lo);
                s = __builtin_amdgcn_sdot4((int)x, 0x01010101, s, false);
                u = __builtin_amdgcn_sdot4((int)x, j0 | ((j0 + 1) << 8) | ((j0 + 2) << 16) | ((j0 + 3) << 24), u, false);
            }
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
        get_mfma(P);
        if (prev) md5_block(Wa);
        weak_mfma();
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
    int32_t hs = 0, hu = 0;  // line 0 before the chunk
    edge_sums(0, true, hs, hu);
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
    int32_t ts = 0, tj = 0;  // line nst after the chunk
    edge_sums((int)(nst & 1), false, ts, tj);
    {
        const uint64_t bits = ((uint64_t)B + 4) * 8;
        uint32_t m[16] = {seed, 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, (uint32_t)bits, (uint32_t)(bits >> 32)};
        md5_compress(st, m);
    }
    int32_t s1, uu;
    {
        const uint32_t nl = nst + 1;  // lines summed by the MFMAs
        int32_t s1g[4], ug[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            Racc[g] += acc[g][0];
            s1g[g] = acc[g][0];
            ug[g] = (int32_t)(128u * (nl * (uint32_t)acc[g][0] - (uint32_t)Racc[g])) + acc[g][1];
        }
        const int src = mfma_pi_inv(l & 15);
        int32_t t1[4], tu[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            t1[g] = __shfl(s1g[g], src, 64);
            tu[g] = __shfl(ug[g], src, 64);
        }
        const int gs = l >> 4;
        s1 = gs == 0 ? t1[0] : gs == 1 ? t1[1] : gs == 2 ? t1[2] : t1[3];
        uu = gs == 0 ? tu[0] : gs == 1 ? tu[1] : gs == 2 ? tu[2] : tu[3];
    }
    // lines -> chunk: S = S_lines - head - tail; sum over the chunk of (i' - a) x' with i' the line-space index
    const uint32_t S = (uint32_t)s1 - (uint32_t)hs - (uint32_t)ts;
    const uint32_t Ui = (uint32_t)uu - (uint32_t)hu - (128u * nst * (uint32_t)ts + (uint32_t)tj) - a * S;
    const uint32_t c = c0 + l;
    const int32_t s2 = (int32_t)(B * S - Ui);
    weak_out[c] = (int32_t)((S & 0xFFFFu) | ((uint32_t)s2 << 16));
    store_digest(strong_out + (size_t)c * dl, st, dl);
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
            block_sums_pipe_body<8, true, true, 0, false, true>(
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
// chunks 3.70-3.75 ms against 3.33 ms without it.
template <int TAIL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(RSH_K1_SHIFT_VGPR))) void block_sums_seg_kernel(
    const K1Seg* __restrict__ segs, uint32_t nseg, const K1Tail* __restrict__ tails, uint32_t ntail, uint32_t B,
    uint32_t dl, uint32_t seed, uint32_t ngf, const int* never) {
    if (blockIdx.x >= nseg) {
        const uint32_t tw = blockIdx.x - nseg, ngw = (ngf + 63u) / 64u;
        if (tw < ngw) {
            block_sums_pipe_body<8, true, true, 0, false, true>(nullptr, B, dl, seed, nullptr, nullptr, never, -1,
                                                               nullptr, 0, 0, 0xFFFFFFFFu, tails + 64u * tw,
                                                               min(64u, ngf - 64u * tw));
            return;
        }
        const uint32_t i = ngf + (tw - ngw) * 64u + threadIdx.x;
        if (i < ntail) {
            const K1Tail t = tails[i];
            if constexpr (TAIL == 0) lane_chunk_sums<2, 4, false>(t.data, t.n, B, t.c, dl, seed, t.weak, t.strong);
            else if constexpr (TAIL == 1) lane_chunk_sums<0, 4, false>(t.data, t.n, B, t.c, dl, seed, t.weak, t.strong);
            else lane_chunk_sums<16, 4, false>(t.data, t.n, B, t.c, dl, seed, t.weak, t.strong);
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
#ifdef RSH_KBENCH
    // tail lanes (kbench A/B: RSH_K1_TAIL=1 (production) dword loads + funnel, 0 wide aligned loads + a per-lane
    // select, 2 plain unaligned dwordx4).  2047 coalesced waves + one tail wave of 64 chunks at offset 1:
    // 3.70-3.75 / 4.13-4.19 / 4.19-4.28 ms (3.33 ms without the tail wave)
    const char* tm = getenv("RSH_K1_TAIL");
    const int mode = tm ? atoi(tm) : 1;
    if (mode == 2) {
        hipLaunchKernelGGL(block_sums_seg_kernel<2>, dim3(waves), dim3(64), lb, s, d_segs, nseg, d_tails, ntail, B, dl,
                           seed_word, ngf, never);
        return hipGetLastError();
    }
    if (mode == 0) {
        hipLaunchKernelGGL(block_sums_seg_kernel<0>, dim3(waves), dim3(64), lb, s, d_segs, nseg, d_tails, ntail, B, dl,
                           seed_word, ngf, never);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(block_sums_seg_kernel<1>, dim3(waves), dim3(64), lb, s, d_segs, nseg, d_tails, ntail, B, dl,
                       seed_word, ngf, never);
    return hipGetLastError();
}


#ifdef RSH_KBENCH
__global__ void block_sums_direct_kernel(const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed,
                                         int32_t* __restrict__ weak_out, uint8_t* __restrict__ strong_out,
                                         const int* abort_flag, int abort_gen);  // device_kbench.inc
template <int S>
__global__ void block_sums_dma_kernel(const uint8_t* __restrict__ data, uint32_t B, uint32_t dl, uint32_t seed,
                                      int32_t* __restrict__ weak_out, uint8_t* __restrict__ strong_out);  // device_kbench.inc
// MD5 step form of the coalesced K1 A/Bs: 0 compiler, 1 one asm statement per step, 2 generated blocks
// (tools/gen_md5_asm.py; the production pipelined K1 uses 2)
constexpr int kMd5Form = 2;
#endif
constexpr uint32_t kCUs = 256;            // MI355X compute units
constexpr uint32_t kLdsPerCU = 160 * 1024; // bytes

// Dynamic LDS above 64 KiB must be enabled per kernel.
template <class K>
void allow_full_lds(K kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kLdsPerCU);
}

// variant: -1 = production choice (19: the pipelined K1 with its tail and shift forms, the coalesced kernel above
// B = 128 KiB, the per-lane kernel for other shapes).  The other variants exist in the kbench build only
// (RSH_KBENCH): 0..2 per-lane (NT PF4, plain PF4, NT PF8); 3..6 coalesced (D=2 NT, D=3 NT, D=2 plain, D=4 NT),
// and the numbered A/Bs below.  Non-coalesced variants handle every chunk shape.
#ifdef RSH_KBENCH
// RSH_K1_PIN_ALL=0 (kbench A/B): K1 launches of more than 2048 waves (single and batched) without the occupancy
// pin -- the coalesced kernel for single files, the unpinned pipelined instantiation for batches
static bool pin_all() {
    static const bool v = !(getenv("RSH_K1_PIN_ALL") && atoi(getenv("RSH_K1_PIN_ALL")) == 0);
    return v;
}
static bool batch_pin() { return pin_all(); }
#else
static bool pin_all() { return true; }
#endif

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

#ifndef RSH_KBENCH
static
#endif
hipError_t launch_block_sums_variant(int variant, const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks,
                                     uint32_t dl, uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong,
                                     hipStream_t s, const int* abort_flag, int abort_gen) {
    if (nchunks == 0) return hipSuccess;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(d_data);
    if (variant < 0) variant = 19;  // coalesced, 2 stages in flight, weak sums on the matrix pipe
#ifdef RSH_KBENCH
    if (variant == 3000 || variant == 3001 || variant == 3002) {  // kbench A/B: the per-lane path at any base
        if (variant == 3002)
            hipLaunchKernelGGL((block_sums_kernel<2, 4, false>), dim3((nchunks + 63) / 64), dim3(64), 0, s, d_data, n,
                               B, nchunks, dl, seed_word, d_weak, d_strong, 0u);
        else if (variant == 3000)
            hipLaunchKernelGGL((block_sums_kernel<16, 4, false>), dim3((nchunks + 63) / 64), dim3(64), 0, s, d_data, n,
                               B, nchunks, dl, seed_word, d_weak, d_strong, 0u);
        else
            hipLaunchKernelGGL((block_sums_kernel<0, 4, false>), dim3((nchunks + 63) / 64), dim3(64), 0, s, d_data, n,
                               B, nchunks, dl, seed_word, d_weak, d_strong, 0u);
        return hipGetLastError();
    }
#endif
    uint32_t c_first = 0;
    const bool deep = variant == 4 || variant == 6 || variant == 7 || variant == 9 || variant == 10 ||
                      variant == 11 || variant == 12 || variant == 14 || variant == 15 || variant == 16 ||
                      variant == 18 || variant == 21 || variant >= 50;  // D >= 3 variants need nst >= 2D = 6 (8 for D = 4)
    // The pipelined K1 also runs at base addresses that are not 16-B aligned (the phase-shifted speculation
    // starts at src + s for any s): its dwordx4 buffer loads then straddle 16-B boundaries, which gfx950
    // serves in its unaligned access mode (bit-exact against the oracle at offsets 0..15,
    // test_k1_unaligned_base).  Option k1_unaligned = 0 (test) sends such bases to the per-lane kernel instead.
    const bool unaligned_ok = opt(OPT_K1_UNALIGNED) != 0;
    // A base that is not 128-B aligned goes to the line-aligned shift kernel when the lines it reads around the
    // data -- a bytes before it, up to 128 - a after the last full wave -- lie in the same allocation (option
    // k1_shift = 0, test: the pipelined kernel at the unaligned base, its path when the lines do not fit).
    if (variant == 19 && (addr % 128) != 0 && (B % 128) == 0 && (B >> 7) >= 4 && (B >> 7) <= 1024 && abort_flag &&
        opt(OPT_K1_SHIFT) != 0) {
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
    if (variant >= 3 && (B % 128) == 0 && (B >> 7) >= (deep ? 8u : 4u) && ((addr % 16) == 0 || unaligned_ok)) {
        const uint32_t nfullc = (uint32_t)std::min<int64_t>(n / B, nchunks);  // chunks with L == B
        const uint32_t waves = nfullc / 64;
        const uint32_t nst = B >> 7;
        const size_t wave_lds = 64 * 9 * sizeof(uint4);
#ifdef RSH_KBENCH
        // LDS per workgroup chosen so that the dispatcher can place at most ceil(groups / CUs) groups
        // on a CU: every SIMD then holds the same number of equal-work waves (no stacking imbalance).
        auto lds_for = [&](uint32_t groups, uint32_t waves_per_group) -> size_t {
            const uint32_t per_cu = std::max<uint32_t>(1, (groups + kCUs - 1) / kCUs);
            size_t bytes = (size_t)kLdsPerCU / per_cu;
            bytes &= ~(size_t)255;
            return std::max(bytes, wave_lds * waves_per_group);
        };
        if ((variant == 7 || variant == 8) && waves >= 4) {
            const uint32_t groups = waves / 4;
            const size_t lb = lds_for(groups, 4);
            if (variant == 8) {
                allow_full_lds(block_sums_coalesced_kernel<2, false, 4>);
                hipLaunchKernelGGL((block_sums_coalesced_kernel<2, false, 4>), dim3(groups), dim3(256), lb, s, d_data,
                                   B, dl, seed_word, d_weak, d_strong);
            } else {
                allow_full_lds(block_sums_coalesced_kernel<3, false, 4>);
                hipLaunchKernelGGL((block_sums_coalesced_kernel<3, false, 4>), dim3(groups), dim3(256), lb, s, d_data,
                                   B, dl, seed_word, d_weak, d_strong);
            }
            c_first = groups * 256;
            variant = 0;
        } else
#endif
        if (waves > 0) {
#ifdef RSH_KBENCH
            const size_t lb = variant == 9 ? lds_for(waves, 1) : wave_lds;
            switch (variant) {
                case 3:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true>), dim3(waves), dim3(64), lb, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
                    break;
                case 5:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, false>), dim3(waves), dim3(64), lb, s, d_data,
                                       B, dl, seed_word, d_weak, d_strong);
                    break;
                case 6:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<4, true>), dim3(waves), dim3(64), lb, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
                    break;
                case 13:
                    hipLaunchKernelGGL((block_sums_dma_kernel<2>), dim3(waves), dim3(64), 2 * 512 * 16, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
                    break;
                case 14:
                    hipLaunchKernelGGL((block_sums_dma_kernel<3>), dim3(waves), dim3(64), 3 * 512 * 16, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
                    break;
                case 15:
                    hipLaunchKernelGGL((block_sums_dma_kernel<4>), dim3(waves), dim3(64), 4 * 512 * 16, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
                    break;
                case 18:
                    if (nst <= 1024) {
                        hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true, 1, 0, false, true>), dim3(waves), dim3(64),
                                           lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    } else {
                        hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true>), dim3(waves), dim3(64), lb, s, d_data,
                                           B, dl, seed_word, d_weak, d_strong);
                    }
                    break;
                case 19:
#else
            const size_t lb = wave_lds;
#endif
                    // the pipelined K1 at any wave count (occupancy pinned to 2 waves/SIMD; beyond 2048 waves they
                    // run in rounds): measured 3.19 vs 3.96 ms for 16 GiB at B = 64 KiB (4096 waves) against the
                    // unpinned instantiation, and ahead of the coalesced kernel at every size
                    if (nst <= 1024 && nst >= 4 && abort_flag && (waves <= 2 * 4 * kCUs || pin_all())) {
                        const uint32_t tail_waves = (nchunks - 64 * waves + 63) / 64;  // in the same launch
                        // the partial last wave's full chunks gathered into a coalesced wave when that adds no
                        // wave or every wave still fits the chip's slots (2 per SIMD)
                        const uint32_t tail_full = nfullc - 64 * waves, tail_short = nchunks - nfullc;
                        const uint32_t gwaves = (tail_full + 63) / 64 + (tail_short + 63) / 64;
                        if (tail_full > 0 && tail_gather_on() &&
                            (gwaves == tail_waves || waves + gwaves <= 2 * 4 * kCUs)) {
                            k1_launch(block_sums_pipe_tailg_kernel<true>, dim3(waves + gwaves), dim3(64),
                                      (uint32_t)(2 * wave_lds), s, d_data, B, dl, seed_word, d_weak, d_strong,
                                      abort_flag, abort_gen, n, nchunks, waves, tail_full);
                            return hipGetLastError();
                        }
                        k1_launch(block_sums_pipe_kernel<8, true, true>, dim3(waves + tail_waves), dim3(64),
                                  (uint32_t)(2 * wave_lds), s, d_data, B, dl, seed_word, d_weak, d_strong, abort_flag,
                                  abort_gen, nullptr, n, nchunks, waves);
                        return hipGetLastError();
                    }
#ifdef RSH_KBENCH
                    else if (nst <= 1024 && nst >= 4 && (waves <= 2 * 4 * kCUs || pin_all())) {
                        hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true>), dim3(waves), dim3(64), 2 * wave_lds,
                                           s, d_data, B, dl, seed_word, d_weak, d_strong);
                    } else if (nst <= 1024 && abort_flag && waves <= 2 * 4 * kCUs) {
                        hipLaunchKernelGGL(
                            (block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, true, kMd5Form, true>),
                            dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong, abort_flag,
                            abort_gen);
                    } else if (nst <= 1024 && abort_flag) {
                        hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, true>),
                                           dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong,
                                           abort_flag, abort_gen);
                    } else if (nst <= 1024 && waves <= 2 * 4 * kCUs) {
                        hipLaunchKernelGGL(
                            (block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, kMd5Form, true>),
                            dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    } else if (nst <= 1024) {
                        hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true>), dim3(waves), dim3(64),
                                           lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    }
#endif
                    else {  // B > 128 KiB (the Generator of a file above 2^34 bytes, config 3): the coalesced K1
                        hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true>), dim3(waves), dim3(64), lb, s, d_data,
                                           B, dl, seed_word, d_weak, d_strong);
                    }
#ifdef RSH_KBENCH
                    break;
                case 20:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, false>), dim3(waves),
                                       dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 21:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true, 1, 0, false, true, false>), dim3(waves),
                                       dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 24:  // A/B: production with the compiler's MD5 step form
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 0, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 25:  // A/B: one asm statement per MD5 step
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 30:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 3, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 31:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 4, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 32:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 1, false, true, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 33:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 3, false, true, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 34:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 3, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 35:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 4, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 36:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, true, false, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 37:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 5, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 38:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 6, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 39:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 5, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 40:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 6, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 41:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, true, false, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 42:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 7, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 43:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 0, false, true, true, false, 8, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 44:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 7, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 45:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 8, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 50:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 0>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 51:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<1, false, true, 0>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 52:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 1>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 53:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<1, false, true, 1>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 54:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, false, 0>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 61:  // A/B: MD5 steps with a + m + K as one v_add3_u32 (K in VGPRs), abortable form
                    hipLaunchKernelGGL(block_sums_pipe_k3_kernel, dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 62:  // A/B: MD5 steps with a + m + K as one v_add3_u32, K from an SGPR (s_mov per step), abortable
                    hipLaunchKernelGGL((block_sums_pipe_kernel<10, true, true>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 66:  // A/B: weak sums from the MD5 words in registers (no MFMA-operand LDS reads), abortable
                    hipLaunchKernelGGL((block_sums_pipe_weakw_kernel), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 67:  // A/B: round 3's production K1 (weak-sum MFMA operands from LDS), abortable
                    hipLaunchKernelGGL((block_sums_pipe_ldsw_kernel), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 68:  // A/B: no LDS -- per-lane loads into registers, weak sums from the MD5 words
                    hipLaunchKernelGGL(block_sums_direct_kernel, dim3(waves), dim3(64), 0, s, d_data, B, dl, seed_word,
                                       d_weak, d_strong, never_word(), -1);
                    break;
                case 64:  // ... without the s_nop after each step
                    hipLaunchKernelGGL((block_sums_pipe_kernel<12, true, true>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 65:  // ... an s_nop after every other step
                    hipLaunchKernelGGL((block_sums_pipe_kernel<13, true, true>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 63:  // ... 16 steps per asm statement
                    hipLaunchKernelGGL((block_sums_pipe_kernel<11, true, true>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 58:  // diagnostics (wrong results): the production abortable K1 on synthetic stage data, no
                          // global loads -- its s_waitcnt time is the LDS / abort-word share (PMC attribution)
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, true, true, 1>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong, never_word(), -1);
                    break;
                case 56:  // A/B: the plain kernel with s_sleep 1 / s_sleep 4 per 2 stages
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 6>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 57:
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 7>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 55:  // A/B: the plain kernel with the abortable kernel's lgkmcnt(0) drain per 2 stages
                    hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 5>), dim3(waves), dim3(64), 2 * wave_lds, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 26:  // diagnostics (wrong results): synthetic data, no weak-sum MFMAs
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 3, false, true, true, false, 2, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 27:  // ... and no LDS transpose, MD5 forms 2 / 1 / 0
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 2, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 28:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 1, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 29:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 4, false, true, true, false, 0, true>),
                                       dim3(waves), dim3(64), lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 22:  // diagnostic: compute only (synthetic stage data), production instantiation otherwise
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 1, false, true, true, false, 2, true>), dim3(waves), dim3(64),
                                       lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 23:  // diagnostic: loads + transpose + weak sums, no MD5
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, true, 1, 2, false, true, true, false, 2, true>), dim3(waves), dim3(64),
                                       lb, s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 16:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true, 1, 0, true>), dim3(waves), dim3(64), lb, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 17:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<2, false, 1, 0, true>), dim3(waves), dim3(64), lb,
                                       s, d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 10:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, false, 1, 1>), dim3(waves), dim3(64), lb, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 11:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, false, 1, 2>), dim3(waves), dim3(64), lb, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 12:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<4, false, 1, 2>), dim3(waves), dim3(64), lb, s,
                                       d_data, B, dl, seed_word, d_weak, d_strong);
                    break;
                case 9:
                    allow_full_lds(block_sums_coalesced_kernel<3, false>);
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, false>), dim3(waves), dim3(64), lb, s, d_data,
                                       B, dl, seed_word, d_weak, d_strong);
                    break;
                default:
                    hipLaunchKernelGGL((block_sums_coalesced_kernel<3, true>), dim3(waves), dim3(64), lb, s, d_data, B,
                                       dl, seed_word, d_weak, d_strong);
            }
#endif
            c_first = waves * 64;
        }
        variant = 0;
    }
    if (c_first >= nchunks) return hipGetLastError();
    const uint32_t rest = nchunks - c_first;
    const dim3 block(64);
    const dim3 grid((rest + 63) / 64);
    if ((B % 16) == 0 && (addr % 16) == 0) {
#ifdef RSH_KBENCH
        if (variant == 1)
            hipLaunchKernelGGL((block_sums_kernel<16, 4, false>), grid, block, 0, s, d_data, n, B, nchunks, dl,
                               seed_word, d_weak, d_strong, c_first);
        else if (variant == 2)
            hipLaunchKernelGGL((block_sums_kernel<16, 8, true>), grid, block, 0, s, d_data, n, B, nchunks, dl,
                               seed_word, d_weak, d_strong, c_first);
        else
#endif
            hipLaunchKernelGGL((block_sums_kernel<16, 4, true>), grid, block, 0, s, d_data, n, B, nchunks, dl,
                               seed_word, d_weak, d_strong, c_first);
    } else if ((B % 4) == 0 && (addr % 4) == 0) {
        hipLaunchKernelGGL((block_sums_kernel<4, 2>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word, d_weak,
                           d_strong, c_first);
    } else {
        hipLaunchKernelGGL((block_sums_kernel<0, 4, false>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong, c_first);
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
// one line for every wave) made the launch 27.9 ms.  RSH_K1_PLAIN=1 (kbench A/B) launches the plain one.
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
#ifdef RSH_KBENCH
static bool plain_k1() {
    static const bool v = getenv("RSH_K1_PLAIN") && atoi(getenv("RSH_K1_PLAIN")) != 0;
    return v;
}
#else
static bool plain_k1() { return false; }
#endif

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
        block_sums_pipe_body<8, true, true, 0, false, true>(g.data, g.B, g.dl, seed, g.weak, g.strong,
                                                           g.abort ? g.abort : abort_flag, abort_gen, nullptr, 0, 0,
                                                           0xFFFFFFFFu, nullptr, g.count);
        return;
    }
    block_sums_pipe_body<8, true, true, 0, true>(nullptr, 0u, 0u, seed, nullptr, nullptr, abort_flag, abort_gen, groups);
}
#ifdef RSH_KBENCH
#include "device_kbench.inc"
#else
static bool batch_quad() { return false; }
#endif

hipError_t launch_block_sums_batch(const K1Group* d_groups, uint32_t ngroups, const K1Lane* d_lanes, uint32_t nlanes,
                                   int lane_align, uint32_t seed_word, hipStream_t s, const int* abort_flag,
                                   int abort_gen, bool partial) {
    const size_t lb = 2 * 64 * 9 * sizeof(uint4);
    static const bool quad = batch_quad();
    if (!abort_flag && !plain_k1() && (abort_flag = never_word()) != nullptr) abort_gen = -1;  // see never_word
    // partial groups, or lanes beside groups: one launch (RSH_K1_GATHER=0: the lanes as a second launch)
    if (partial || (tail_gather_on() && !quad && nlanes > 0 && ngroups > 0)) {
        if (!abort_flag && (abort_flag = never_word()) != nullptr) abort_gen = -1;
        if (!abort_flag || quad) return hipErrorInvalidValue;  // the planner makes no partial group for these
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
#ifdef RSH_KBENCH
    if (ngroups > 0 && quad) {
        const hipError_t e = launch_block_sums_batch_quad(d_groups, ngroups, seed_word, s, abort_flag, abort_gen);
        if (e != hipSuccess) return e;
        ngroups = 0;
    }
#endif
    if (ngroups > 0) {
#ifdef RSH_KBENCH
        if (abort_flag && batch_pin())
            hipLaunchKernelGGL((block_sums_pipe_kernel<8, true, true, 0, true>), dim3(ngroups), dim3(64), lb, s,
                               nullptr, 0u, 0u, seed_word, nullptr, nullptr, abort_flag, abort_gen, d_groups);
        else if (abort_flag)
            hipLaunchKernelGGL((block_sums_pipe_kernel<8, true, false, 0, true>), dim3(ngroups), dim3(64), lb, s,
                               nullptr, 0u, 0u, seed_word, nullptr, nullptr, abort_flag, abort_gen, d_groups);
        else if (batch_pin())
            hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, true, 0, true>), dim3(ngroups), dim3(64), lb, s,
                               nullptr, 0u, 0u, seed_word, nullptr, nullptr, nullptr, 0, d_groups);
        else
            hipLaunchKernelGGL((block_sums_pipe_kernel<8, false, false, 0, true>), dim3(ngroups), dim3(64), lb, s,
                               nullptr, 0u, 0u, seed_word, nullptr, nullptr, nullptr, 0, d_groups);
#else
        if (!abort_flag) return hipErrorOutOfMemory;  // never_word() failed: no uncached word for the pinned K1
        hipLaunchKernelGGL((block_sums_pipe_kernel<8, true, true, 0, true>), dim3(ngroups), dim3(64), lb, s, nullptr,
                           0u, 0u, seed_word, nullptr, nullptr, abort_flag, abort_gen, d_groups);
#endif
    }
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
#ifdef RSH_KBENCH
    // RSH_K1_VARIANT (kbench A/B) replaces the production variant for non-abortable launches
    static const int forced = getenv("RSH_K1_VARIANT") ? atoi(getenv("RSH_K1_VARIANT")) : -1;
#else
    constexpr int forced = -1;
#endif
    if (!abort_flag && forced < 0 && !plain_k1() && (abort_flag = never_word()) != nullptr) abort_gen = -1;
    return launch_block_sums_variant(abort_flag ? -1 : forced, d_data, n, B, nchunks, dl, seed_word, d_weak, d_strong, s, abort_flag,
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

// ------------------------------------------------------------------------------------------------
// Probe table (distinct weak keys).  Slot = (1 << 32) | key; 0 = empty.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t slot_hash(uint32_t key) {
    uint32_t h = key * 0x9E3779B1u;
    return h ^ (h >> 15);
}

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
// Weighted byte sums over a range: S1 = sum x_j, S2 = sum (j - org) * x_j (signed bytes, mod 2^32),
// accumulated by one workgroup with 16-byte loads where the range is 16-aligned.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void dword_sums(uint32_t w, uint32_t rel, int32_t& s1, int32_t& s2) {
    const int32_t a = __builtin_amdgcn_sdot4((int)w, 0x01010101, 0, false);
    s1 += a;
    s2 += (int32_t)(rel * (uint32_t)a) + __builtin_amdgcn_sdot4((int)w, 0x03020100, 0, false);
}

// Sums of bytes [lo, hi) (clipped to [0, n)) relative to origin org, over all threads of the block.
// Returns this thread's partial; the caller reduces.
__device__ __forceinline__ void range_sums(const uint8_t* __restrict__ x, int64_t n, int64_t lo, int64_t hi, int64_t org,
                                           int32_t& s1, int32_t& s2) {
    if (hi > n) hi = n;
    if (lo >= hi) return;
    const int t = threadIdx.x, T = blockDim.x;
    int64_t a16 = (lo + 15) & ~(int64_t)15;
    if (a16 > hi) a16 = hi;
    const int64_t b16 = a16 + ((hi - a16) & ~(int64_t)15);
    for (int64_t j = lo + t; j < a16; j += T) {  // unaligned head
        const int32_t v = sbyte(x[j]);
        s1 += v;
        s2 += (int32_t)((uint32_t)(j - org) * (uint32_t)v);
    }
    // 64-B pieces per lane, eight 16-B loads in flight before any use (a 128 KiB window in a few round
    // trips instead of one per 4 KiB: these single-workgroup reductions sit on the resolver's latency path)
    int64_t j = a16 + 64 * (int64_t)t;
    for (; j + 64 * (int64_t)T + 64 <= b16; j += 128 * (int64_t)T) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const uint4*>(x + j + 16 * k);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 + k] = *reinterpret_cast<const uint4*>(x + j + 64 * (int64_t)T + 16 * k);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t rel = (uint32_t)(j + (k >= 4 ? 64 * (int64_t)T : 0) + 16 * (k & 3) - org);
            dword_sums(v[k].x, rel, s1, s2);
            dword_sums(v[k].y, rel + 4, s1, s2);
            dword_sums(v[k].z, rel + 8, s1, s2);
            dword_sums(v[k].w, rel + 12, s1, s2);
        }
    }
    for (; j < b16; j += 64 * (int64_t)T) {  // remaining 64-B pieces (the last may be 16..48 B)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (j + 16 * k >= b16) break;
            const uint4 v = *reinterpret_cast<const uint4*>(x + j + 16 * k);
            const uint32_t rel = (uint32_t)(j + 16 * k - org);
            dword_sums(v.x, rel, s1, s2);
            dword_sums(v.y, rel + 4, s1, s2);
            dword_sums(v.z, rel + 8, s1, s2);
            dword_sums(v.w, rel + 12, s1, s2);
        }
    }
    for (int64_t j = b16 + t; j < hi; j += T) {  // tail
        const int32_t v = sbyte(x[j]);
        s1 += v;
        s2 += (int32_t)((uint32_t)(j - org) * (uint32_t)v);
    }
}

template <int NV>
__device__ __forceinline__ void block_reduce(int32_t (&v)[NV], int32_t* sh /* NV * blockDim / 64 */) {
    const int t = threadIdx.x, nw = blockDim.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int32_t x = v[i];
        for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
        v[i] = x;
    }
    __syncthreads();
    if ((t & 63) == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) sh[i * nw + (t >> 6)] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int32_t x = 0;
        for (int w = 0; w < nw; ++w) x += sh[i * nw + w];
        v[i] = x;
    }
    __syncthreads();
}

// exclusive scan over the block's threads (thread order), NV values at once
template <int NV>
__device__ __forceinline__ void block_exscan(int32_t (&v)[NV], int32_t* sh /* NV * blockDim / 64 */) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = blockDim.x >> 6;
    int32_t incl[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int32_t x = v[i];
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        incl[i] = x;
    }
    __syncthreads();
    if (lane == 63)
#pragma unroll
        for (int i = 0; i < NV; ++i) sh[i * nw + wv] = incl[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int32_t base = 0;
        for (int w = 0; w < wv; ++w) base += sh[i * nw + w];
        v[i] = base + incl[i] - v[i];
    }
    __syncthreads();
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
constexpr int PROBE_THREADS = 256;
constexpr int PROBE_PPT = 16;
static_assert(PROBE_TILE == PROBE_THREADS * PROBE_PPT, "tile = threads x positions per thread");

__device__ __forceinline__ int32_t roll_sub(int32_t cs, int32_t w, int32_t x) {  // Rolling.java:56-60
    const uint32_t lo = ((uint32_t)cs & 0xFFFFu) - (uint32_t)x;
    const uint32_t hi = ((uint32_t)cs >> 16) - (uint32_t)__mul24(w, x);  // (w <= B <= 2^17: a full-rate 24-bit multiply)
    return (int32_t)((lo & 0xFFFFu) | (hi << 16));
}
__device__ __forceinline__ int32_t roll_add(int32_t cs, int32_t x) {  // Rolling.java:25-29
    const uint32_t lo = ((uint32_t)cs & 0xFFFFu) + (uint32_t)x;
    const uint32_t hi = ((uint32_t)cs >> 16) + lo;
    return (int32_t)((lo & 0xFFFFu) | (hi << 16));
}

// 16 bytes at p (zero outside [0, n)) as 4 little-endian words: bytes stay packed in 4 VGPRs
__device__ __forceinline__ void load16(const uint8_t* __restrict__ x, int64_t n, int64_t p, uint32_t (&w)[4]) {
    if (p >= 0 && p + 16 <= n && ((reinterpret_cast<uintptr_t>(x + p) & 15) == 0)) {
        const uint4 q = *reinterpret_cast<const uint4*>(x + p);
        w[0] = q.x;
        w[1] = q.y;
        w[2] = q.z;
        w[3] = q.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (p + i < n && p + i >= 0) w[i >> 2] |= (uint32_t)x[p + i] << (8 * (i & 3));
    }
}
__device__ __forceinline__ int32_t sbyte_of(const uint32_t (&w)[4], int i) {
    return (int32_t)(int8_t)(uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

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

// grid (1 + 16, nreq): block 0 computes T(p) and the key, blocks 1..16 copy the window.
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
    hipLaunchKernelGGL(hit_window_kernel, dim3(1 + 16 * HIT_WINDOWS, (uint32_t)nreq), dim3(256), 0, s, files, ivs, req);
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
            int32_t R = (int32_t)(((s1 + I.e_lo) & 0xFFFFu) | ((s2 + ehi) << 16));
#pragma unroll 1
            for (int grp = 0; grp < PROBE_LONG_PPL / 16; ++grp) {  // 16 positions at a time (bytes re-read: L1)
                uint32_t wa[4], wb[4];
                load16(data, n, p0 + 16 * grp, wa);
                load16(data, n, p0 + B + 16 * grp, wb);
                uint32_t key[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {  // full windows throughout: w = B, the add always follows
                    key[i] = (uint32_t)R;
                    R = roll_add(roll_sub(R, (int32_t)B, sbyte_of(wa, i)), sbyte_of(wb, i));
                }
                const uint32_t valid = probe_valid16(p0 + 16 * grp, I.a, I.b < q1 ? I.b : q1);
                if (valid) probe_check16(F, table, nsmall, key, valid, p0 + 16 * grp);
            }
            if (t == PROBE_THREADS - 1) {  // R(p0 + 64) less E there: the next sub-segment's anchor T
                const int64_t pn = p0 + PROBE_LONG_PPL;
                const uint32_t en = I.e_hi + I.e_lo * (uint32_t)(clampB(pn) - clampB(I.anchor));
                const uint32_t r = (uint32_t)R;
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

constexpr int CHAIN_HELP_TILES = 4;   // a walk gets helpers once it has searched this many tiles
constexpr int CHAIN_HELP_LEAD = 64;   // a helper stays with its file while the map leads the walk by fewer segments
// A helper workgroup: while some walk that has searched CHAIN_HELP_TILES tiles is still running, take the next
// unmapped segment of the one whose map leads it least (its own current file while the lead is short: the key set is
// built per file) -- never the segment the walk is in, which it will finish first -- and map it tile by tile,
// stopping when the walk ends or has passed the tile.  While walks are running that have not searched that far yet it
// sleeps and looks again; once no mappable walk is running it leaves.  No walk ever waits for a helper: a walk reads
// a map word only when it carries this launch's generation, and searches the tile itself otherwise.  (A helper waits
// only for walks of its own launch, whose workgroups precede it in dispatch order.)
__device__ __attribute__((noinline)) void chain_help(const ChainFile* __restrict__ files, int nfiles, uint32_t gen,
                                                     ChainHelp* help, uint2* ck, int32_t* ck_full,
                                                     int32_t* sh, int32_t (*s_seg)[4], unsigned long long* s_best,
                                                     int32_t* s_word, int32_t* s_live) {
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
            if (tiles < CHAIN_HELP_TILES) continue;
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
            __builtin_amdgcn_s_sleep(64);  // walks still short of CHAIN_HELP_TILES tiles: look again shortly
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
            const int64_t tb = (int64_t)wall_clock64();
            F = files[f];
            chain_kset_build(kset, F.table_weak, F.C);
            if (t == 0) {
                atomicAdd((unsigned long long*)&h->t_kset, (unsigned long long)((int64_t)wall_clock64() - tb));
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
                atomicMin((unsigned long long*)&h->t_first, (unsigned long long)wall_clock64());
            }
        }
    }
    if (t == 0 && cur >= 0) atomicSub(&help[cur].nhelp, 1);
}

__global__ __launch_bounds__(CHAIN_THREADS) void chain_advance_kernel(const ChainFile* __restrict__ files, int phase,
                                                                      int abort_gen, ChainHelp* help, int nfiles) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[4 * CHAIN_THREADS / 64];
    __shared__ int32_t s_hit;                  // first hit in a tile (offset from the tile start), or INT_MAX
    __shared__ uint32_t s_key;                 // its key
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
        chain_help(files, nfiles, (uint32_t)abort_gen, help, s_ck, &s_ck_full, sh, s_seg, &s_best, &s_word, &s_live);
        return;
    }
    // the descriptor by value: it sits in pinned host memory, and a reference would let the compiler re-read its
    // fields across the loop (the event stores may alias it) -- a PCIe round trip each
    const ChainFile F = files[blockIdx.x];
    ChainHelp* const H = (phase == 0 && help != nullptr) ? help + blockIdx.x : nullptr;
    if (H != nullptr && threadIdx.x == 0) chain_st64(&H->t_start, (int64_t)wall_clock64());
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
    if (kset_built) chain_kset_build(kset, F.table_weak, C);
    int32_t pref = out->pref;
    int32_t nev = out->n_ev, status = CHAIN_STOP;
    int64_t lit = out->literal, mat = out->matched, chain_matches = out->chain_matches, events = out->events;
    int32_t tiles = out->tiles, digests = out->digests, poisoned = 0, dead = 0, mapped = out->mapped;
    int32_t first_mapped = out->first_mapped;
    int64_t flushes = out->flushes;
    const int64_t tk0 = (int64_t)wall_clock64();
    int64_t t_tiles = 0, t_check = 0, t_event = 0, t_digest = 0;
    const uint8_t* stale = nullptr;  // poisoned: the cached digest
    uint32_t dg[4] = {0u, 0u, 0u, 0u};  // the window's digest at the current event (poisoned: the stale one)
    int64_t clear_to = -1;            // stopped at a flush point: no candidate in [s, clear_to]
    int32_t why = CHAIN_WHY_NONE;
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
        __syncthreads();
        for (int32_t i = t; i < nev - nev_w; i += CHAIN_THREADS) F.ev[nev_w + i] = s_ev[i];
        nev_w = nev;
        __syncthreads();
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
        const uint8_t flag_k = (!poisoned && k == pref && k < nflags) ? F.flags[k] : (uint8_t)0;
        const int32_t aw_k = (al && k < na) ? F.aw[k] : 0;
        const int32_t tw_pref = (!poisoned && pref < C && k < na) ? F.table_weak[pref] : 0;
        // (1) aligned chain: preferred index == k and source window k carries chunk k's sums
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
                continue;
            }
        }
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
                const int64_t tt0 = (int64_t)wall_clock64();
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
                    if (t == 0) s_hit = 0x7FFFFFFF;
                    if (__syncthreads_and(!need || (uint32_t)(wv >> 32) == map_gen)) {
                        if (need) {
                            const uint32_t bits = (uint32_t)wv & (0xFFFFFFFFu >> (31 - (hi < 31 ? hi : 31))) &
                                                  (0xFFFFFFFFu << lo);
                            if (bits) atomicMin(&s_hit, (int32_t)(pm - q0) + __builtin_ctz(bits));
                        }
                        __syncthreads();
                        const int32_t hoff = s_hit;
                        if (hoff != 0x7FFFFFFF && al_lane && pm == q0 + hoff) s_key = (uint32_t)awl;
                        __syncthreads();
                        if (hoff != 0x7FFFFFFF) {  // the key: the window's true weak sum (synced)
                            p = q0 + hoff;
                            if (p % B == 0) {      // an aligned window: the speculation's sum, loaded above
                                key = s_key;
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
                        t_tiles += (int64_t)wall_clock64() - tt0;
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
                const int64_t tc0 = (int64_t)wall_clock64();
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
                t_check += (int64_t)wall_clock64() - tc0;
                if (my_hit != 0x7FFFFFFF && my_hit == s_hit) s_key = my_key;
                __syncthreads();
                if (s_hit != 0x7FFFFFFF) {
                    p = q0 + s_hit;
                    key = s_key;
                }
                __syncthreads();
                q0 += CHAIN_TILE;
                t_tiles += (int64_t)wall_clock64() - tt0;
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
        const int64_t te0 = (int64_t)wall_clock64();
        ++events;
        const int64_t kp = p / B;
        const bool spec_digest = !poisoned && p % B == 0 && kp < na;
        // the speculation's digest of an aligned window, loaded beside the bucket's slots (it depends only on p)
        // ... and chunk kp's own digest beside it: the candidate of a window that sits where its chunk sat (identical
        // stretches, edited blocks in place) is decided without another round trip
        uint32_t dgk[4] = {0u, 0u, 0u, 0u};
        const bool diag = spec_digest && kp < C;
        if (spec_digest) chain_digest_load(F.as + kp * dl, dl, dg);
        if (diag) chain_digest_load(F.table_strong + kp * dl, dl, dgk);
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
            if (t == 0) s_nbk = cnt;
        }
        __syncthreads();
        if (t == 0) {
            const int32_t cnt = s_nbk;
            for (int i = 1; i < cnt && i < CHAIN_BUCKET_CAP; ++i)  // ascending chunk index (insertion order)
                for (int j = i; j > 0 && s_bk[j - 1] > s_bk[j]; --j) {
                    const int32_t x = s_bk[j];
                    s_bk[j] = s_bk[j - 1];
                    s_bk[j - 1] = x;
                }
        }
        __syncthreads();
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
            const int64_t td0 = (int64_t)wall_clock64();
            chain_window_digest(F.data + p, (uint32_t)B, (uint32_t)dl, F.seed, s_win, s_dig);  // (ends with a barrier)
            md5c = s_dig;
            chain_digest_load(s_dig, dl, dg);
            ++digests;
            t_digest += (int64_t)wall_clock64() - td0;
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
        t_event += (int64_t)wall_clock64() - te0;
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
                        any |= chain_digest_eq_reg(dg, F.table_strong + c * dl, dl) |
                               chain_digest_eq_reg(dg, F.table_strong + c2 * dl, dl);
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
                why = CHAIN_WHY_FLUSHHIT;
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
        out->t_total += (int64_t)wall_clock64() - tk0;
        out->t_tiles += t_tiles;
        out->t_check += t_check;
        out->t_event += t_event;
        out->t_digest += t_digest;
        out->spec_full = phase == 1;
        out->mapped = mapped;
        out->clear_to = clear_to;
        out->why = why;
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
    }
    if (H != nullptr) {  // this walk is over: its helpers stop, and the workgroup helps the walks still searching
        if (t == 0) chain_st(&H->live, 0);
        __syncthreads();
        chain_help(files, nfiles, (uint32_t)abort_gen, help, s_ck, &s_ck_full, sh, s_seg, &s_best, &s_word, &s_live);
    }
}

hipError_t launch_chain_advance(const ChainFile* files, uint32_t nfiles, hipStream_t s, int phase, int abort_gen,
                                ChainHelp* help, uint32_t helpers) {
    if (nfiles == 0) return hipSuccess;
    if (phase != 0 || help == nullptr || nfiles >= (1u << 20)) {  // (helpers pick files by a 20-bit index)
        help = nullptr;
        helpers = 0;
    }
    hipLaunchKernelGGL(chain_advance_kernel, dim3(nfiles + helpers), dim3(CHAIN_THREADS), 0, s, files, phase,
                       abort_gen, help, (int)nfiles);
    return hipGetLastError();
}

// The chunk index of the chain walk: every chunk i of a file as (key << 32) | (i + 1) in an open-addressing table
// (0 = empty); the chunks with one key all lie on that key's probe path before its first empty slot.
// A thread's keys go in groups of CHUNK_INDEX_MLP: the group's first-slot CASes are issued back to back (independent
// atomics, all in flight at once), and only a CAS that found its slot taken walks the probe path (a serial
// CAS-then-next loop keeps one atomic round trip in flight per thread).  Config 4's 2 M chunks on the background
// grid beside the prefix K1: the index now ends inside that launch instead of 0.03 ms after it.
constexpr int CHUNK_INDEX_MLP = 8;
__global__ void chunk_index_kernel(const TableEnt* __restrict__ ents, uint32_t nfiles) {
    const TableEnt e = ents[blockIdx.y];
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
            if (got[j] == 0ull) continue;
            uint32_t hh = (h[j] + 1) & e.mask;
            while (atomicCAS(&e.slots[hh], 0ull, v[j]) != 0ull) hh = (hh + 1) & e.mask;
        }
    }
    (void)nfiles;
}

hipError_t launch_chunk_index(const TableEnt* ents, uint32_t nfiles, int32_t max_keys, hipStream_t s, bool bg) {
    if (nfiles == 0 || max_keys <= 0) return hipSuccess;
    const uint32_t gx = (uint32_t)std::min<int64_t>((max_keys + 255) / 256, bg ? 2 : 64);
    hipLaunchKernelGGL(chunk_index_kernel, dim3(gx, nfiles), dim3(256), 0, s, ents, nfiles);
    return hipGetLastError();
}

__global__ void gather_bytes_kernel(const ScanFile* __restrict__ files, const GatherEnt* __restrict__ ents, uint32_t n,
                                    uint8_t* __restrict__ out) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const GatherEnt e = ents[i];
        out[i] = files[e.file].data[e.p];
    }
}

hipError_t launch_gather_bytes(const ScanFile* files, const GatherEnt* ents, uint32_t n, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_bytes_kernel, dim3((n + 255) / 256), dim3(256), 0, s, files, ents, n, out);
    return hipGetLastError();
}

// Device bytes -> pinned host memory, as a kernel: the runtime's copy path can queue behind a
// co-running speculation launch, a high-priority kernel does not.  Thread t assembles bytes
// [16t, 16t + 16) and writes them with one 16-byte store (dst 16-byte aligned).
__device__ __forceinline__ void copy_piece(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t n,
                                           int64_t o) {
    if (o + 16 <= n) {
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i >> 2] |= (uint32_t)src[o + i] << (8 * (i & 3));
        *reinterpret_cast<uint4*>(dst + o) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (int64_t i = o; i < n; ++i) dst[i] = src[i];
    }
}

__global__ __launch_bounds__(256) void copy_to_host_kernel(const uint8_t* __restrict__ src, int64_t n,
                                                           uint8_t* __restrict__ dst) {
    __builtin_amdgcn_s_setprio(3);
    const int64_t o = 16 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (o < n) copy_piece(src, dst, n, o);
}

hipError_t launch_copy_to_host(const uint8_t* d_src, int64_t n, uint8_t* h_dst, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t threads = (n + 15) / 16;
    hipLaunchKernelGGL(copy_to_host_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, d_src, n, h_dst);
    return hipGetLastError();
}

// The last workgroup of a stamped launch.  No fence per workgroup: on this chip a fence at agent scope writes the
// XCD's L2 back (its L2s are not coherent with each other), and one per workgroup cost the first version ~230 us for
// 2304 workgroups (r5j trace).  Instead every thread waits for its own memory operations (vmcnt also counts stores and
// atomics here), then one thread per workgroup counts the workgroup done with a device atomic; the workgroup that
// completes the count -- its reads of the others' results are device atomics too -- releases at system scope once and
// writes the stamp, which the host polls before it reads what the launch wrote to host memory.
__device__ __forceinline__ bool stamp_arrive(const Stamp& st, bool* sh_last) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) *sh_last = atomicAdd(st.counter, 1u) == gridDim.x * gridDim.y - 1;
    __syncthreads();
    return *sh_last;
}
__device__ __forceinline__ void stamp_write(const Stamp& st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicExch(st.counter, 0u);
        __threadfence_system();
        __hip_atomic_store(st.stamp, st.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(256) void chain_flags_stamped_kernel(const int32_t* __restrict__ wsrc,
                                                                  const uint8_t* __restrict__ ssrc,
                                                                  const int32_t* __restrict__ wbas,
                                                                  const uint8_t* __restrict__ sbas, uint32_t count,
                                                                  uint32_t dl, uint8_t* __restrict__ flags, Stamp st) {
    __shared__ bool last;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < count) {
        bool eq = wsrc[k] == wbas[k];
        for (uint32_t j = 0; j < dl; ++j) eq &= ssrc[(size_t)k * dl + j] == sbas[(size_t)k * dl + j];
        flags[k] = eq ? 1 : 0;
    }
    if (stamp_arrive(st, &last)) stamp_write(st);
}

hipError_t launch_chain_flags_stamped(const int32_t* d_wsrc, const uint8_t* d_ssrc, const int32_t* d_wbas,
                                      const uint8_t* d_sbas, uint32_t count, uint32_t dl, uint8_t* h_flags,
                                      Stamp st, hipStream_t s) {
    hipLaunchKernelGGL(chain_flags_stamped_kernel, dim3(count ? (count + 255) / 256 : 1), dim3(256), 0, s, d_wsrc,
                       d_ssrc, d_wbas, d_sbas, count, dl, h_flags, st);
    return hipGetLastError();
}

// blockIdx.x < nsamp * pieces: piece (blockIdx.x % pieces) of sample window blockIdx.x / pieces; the blocks past them
// copy window 0 to the host, 4 KiB each.
__global__ __launch_bounds__(256) void scan_prep_kernel(ScanPrep P) {
    __shared__ int32_t sh[2 * 4];
    __shared__ bool last;
    const uint32_t b = blockIdx.x, nsum = P.nsamp * P.pieces;
    if (b < nsum) {
        const uint32_t i = b / P.pieces, q = b % P.pieces;
        const int64_t p = P.wins[i] * (int64_t)P.B, w = P.n - p < (int64_t)P.B ? P.n - p : (int64_t)P.B;
        const int64_t plen = ((w + P.pieces - 1) / P.pieces + 15) & ~(int64_t)15;
        const int64_t lo = p + (int64_t)q * plen, hi = lo + plen < p + w ? lo + plen : p + w;
        int32_t v[2] = {0, 0};
        range_sums(P.data, P.n, lo, hi, p, v[0], v[1]);
        block_reduce<2>(v, sh);
        if (threadIdx.x == 0) {
            atomicAdd(&P.scratch[2 * i], v[0]);
            atomicAdd(&P.scratch[2 * i + 1], v[1]);
        }
    } else {
        const int64_t o = 16 * ((int64_t)(b - nsum) * blockDim.x + threadIdx.x);
        if (o < P.w0_len) copy_piece(P.data, P.w0, P.w0_len, o);
    }
    if (!stamp_arrive(P.st, &last)) return;
    for (uint32_t i = threadIdx.x; i < P.nsamp; i += blockDim.x) {
        const int64_t k = P.wins[i], p = k * (int64_t)P.B, w = P.n - p < (int64_t)P.B ? P.n - p : (int64_t)P.B;
        const uint32_t S1 = (uint32_t)atomicExch(&P.scratch[2 * i], 0);
        const uint32_t U = (uint32_t)atomicExch(&P.scratch[2 * i + 1], 0);
        const uint32_t S2 = (uint32_t)w * S1 - U;
        P.out_t[i] = (int32_t)((S1 & 0xFFFFu) | (S2 << 16));
        P.out_w[i] = k < P.C ? P.table_weak[k] : 0;
    }
    stamp_write(P.st);
}

hipError_t launch_scan_prep(const ScanPrep& P, hipStream_t s) {
    const uint32_t copy_blocks = (uint32_t)((P.w0_len + 16 * 256 - 1) / (16 * 256));
    hipLaunchKernelGGL(scan_prep_kernel, dim3(P.nsamp * P.pieces + copy_blocks), dim3(256), 0, s, P);
    return hipGetLastError();
}

// grid (., n): entry blockIdx.y, 16 bytes per thread, grid-strided over the entry's length
__global__ __launch_bounds__(256) void copy_many_kernel(const CopyEnt* __restrict__ ents, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(3);
    const CopyEnt e = ents[blockIdx.y];
    for (int64_t o = 16 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); o < e.len;
         o += 16 * (int64_t)gridDim.x * blockDim.x)
        copy_piece(e.src, e.dst, e.len, o);
}

hipError_t launch_copy_many(const CopyEnt* ents, uint32_t n, int64_t max_len, hipStream_t s, bool bg) {
    if (n == 0 || max_len <= 0) return hipSuccess;
    const int64_t blocks = bg ? 1 : std::min<int64_t>((max_len + 16 * 256 - 1) / (16 * 256), 64);
    hipLaunchKernelGGL(copy_many_kernel, dim3((uint32_t)blocks, n), dim3(256), 0, s, ents, bg ? 0 : 1);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// True weak sums at arbitrary positions (one workgroup per position).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void window_weak_kernel(const ScanFile* __restrict__ files,
                                                          const GatherEnt* __restrict__ ents,
                                                          int32_t* __restrict__ out) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ int32_t sh[2 * 256 / 64];
    const GatherEnt e = ents[blockIdx.x];
    const ScanFile& F = files[e.file];
    const int64_t p = e.p, n = F.n, B = F.B;
    const int64_t w = (n - p < B ? n - p : B);
    int32_t v[2] = {0, 0};
    range_sums(F.data, n, p, p + w, p, v[0], v[1]);
    block_reduce<2>(v, sh);
    if (threadIdx.x == 0) {
        const uint32_t S1 = (uint32_t)v[0];
        const uint32_t S2 = (uint32_t)w * S1 - (uint32_t)v[1];
        const int32_t T = (int32_t)((S1 & 0xFFFFu) | (S2 << 16));
        if (e.by_block) F.aligned_weak[p / B] = T;
        else out[blockIdx.x] = T;
    }
}

hipError_t launch_window_weak(const ScanFile* files, const GatherEnt* ents, uint32_t n, int32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(window_weak_kernel, dim3(n), dim3(256), 0, s, files, ents, out);
    return hipGetLastError();
}

// D dwordx4 loads in flight per thread before their stores; NTL / NTS: non-temporal loads / stores.  The production
// form is <1024, 4, true, true>; the others are kbench A/Bs (KBENCH_GATHER).
template <int T, int D, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void gather_ops_kernel_t(const GatherOp* __restrict__ ops) {
    const GatherOp op = ops[blockIdx.x];
    const uintptr_t d = reinterpret_cast<uintptr_t>(op.dst);
    int64_t head = (int64_t)((16 - (d & 15)) & 15);
    if (head > op.len) head = op.len;
    const int t = threadIdx.x;
    if (t < head) op.dst[t] = op.src[t];
    const int64_t body = (op.len - head) & ~(int64_t)15;
    const uint8_t* __restrict__ s = op.src + head;
    uint8_t* __restrict__ o = op.dst + head;
    if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {  // 16-B aligned source: dwordx4 loads, 4 in flight
        const int64_t step = 16 * (int64_t)T;
        int64_t k = 16 * (int64_t)t;
        for (; k + (D - 1) * step < body; k += D * step) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4 v[D];
#pragma unroll
            for (int u = 0; u < D; ++u) {
                const u32x4* a = reinterpret_cast<const u32x4*>(s + k + u * step);
                if constexpr (NTL) v[u] = __builtin_nontemporal_load(a);
                else v[u] = *a;
            }
#pragma unroll
            for (int u = 0; u < D; ++u) {
                u32x4* a = reinterpret_cast<u32x4*>(o + k + u * step);
                if constexpr (NTS) __builtin_nontemporal_store(v[u], a);
                else *a = v[u];
            }
        }
        for (; k < body; k += step)
            *reinterpret_cast<uint4*>(o + k) = *reinterpret_cast<const uint4*>(s + k);
    } else if ((reinterpret_cast<uintptr_t>(s) & 3) == 0) {  // word-aligned source: four dword loads per store
        for (int64_t k = 16 * (int64_t)t; k < body; k += 16 * (int64_t)blockDim.x) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(s + k);
            *reinterpret_cast<uint4*>(o + k) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    } else {
        for (int64_t k = 16 * (int64_t)t; k < body; k += 16 * (int64_t)blockDim.x) {
            uint32_t q[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 16; ++i) q[i >> 2] |= (uint32_t)s[k + i] << (8 * (i & 3));
            *reinterpret_cast<uint4*>(o + k) = make_uint4(q[0], q[1], q[2], q[3]);
        }
    }
    for (int64_t k = head + body + t; k < op.len; k += blockDim.x) op.dst[k] = op.src[k];
}

hipError_t launch_gather_ops(const GatherOp* ops, uint32_t n, hipStream_t s, int64_t avg_len) {
    if (n == 0) return hipSuccess;
    if (avg_len < (64 << 10)) {  // short ops (a segment's 8 KiB literal tokens and blocks): 256 threads each
        hipLaunchKernelGGL((gather_ops_kernel_t<256, 2, true, true>), dim3(n), dim3(256), 0, s, ops);
        return hipGetLastError();
    }
    // 1024 threads per 1 MiB op (16 waves per CU in flight): 0.754 of the 8 TB/s peak (read + write) against 0.680 for
    // 256 threads, kbench KBENCH_GATHER (profiles/r4/r4e_kbench_gather.log)
    hipLaunchKernelGGL((gather_ops_kernel_t<1024, 4, true, true>), dim3(n), dim3(1024), 0, s, ops);
    return hipGetLastError();
}
#ifdef RSH_KBENCH
hipError_t launch_gather_ops_variant(int v, const GatherOp* ops, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    switch (v) {
        case 1: hipLaunchKernelGGL((gather_ops_kernel_t<256, 8, true, true>), dim3(n), dim3(256), 0, s, ops); break;
        case 2: hipLaunchKernelGGL((gather_ops_kernel_t<512, 4, true, true>), dim3(n), dim3(512), 0, s, ops); break;
        case 3: hipLaunchKernelGGL((gather_ops_kernel_t<256, 4, false, true>), dim3(n), dim3(256), 0, s, ops); break;
        case 4: hipLaunchKernelGGL((gather_ops_kernel_t<256, 4, false, false>), dim3(n), dim3(256), 0, s, ops); break;
        case 5: hipLaunchKernelGGL((gather_ops_kernel_t<512, 8, true, true>), dim3(n), dim3(512), 0, s, ops); break;
        case 6: hipLaunchKernelGGL((gather_ops_kernel_t<1024, 4, true, true>), dim3(n), dim3(1024), 0, s, ops); break;
        default: hipLaunchKernelGGL((gather_ops_kernel_t<256, 4, true, true>), dim3(n), dim3(256), 0, s, ops); break;
    }
    return hipGetLastError();
}
#endif

__global__ void table_insert_many_kernel(const TableEnt* __restrict__ ents, int hi) {
    if (hi) __builtin_amdgcn_s_setprio(3);
    const TableEnt e = ents[blockIdx.y];
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < e.nkeys; i += gridDim.x * blockDim.x) {
        const uint32_t key = (uint32_t)e.keys[i];
        const unsigned long long v = (1ull << 32) | key;
        uint32_t h = slot_hash(key) & e.mask;
        for (uint32_t probes = 0; probes <= e.mask; ++probes) {
            const unsigned long long prev = atomicCAS(&e.slots[h], 0ull, v);
            if (prev == 0ull || prev == v) break;
            h = (h + 1) & e.mask;
        }
    }
}

hipError_t launch_table_insert_many(const TableEnt* ents, uint32_t n, int32_t max_keys, hipStream_t s, bool bg) {
    if (n == 0 || max_keys <= 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<int64_t>((max_keys + 255) / 256, bg ? std::max<uint32_t>(1, kBackgroundGroups / n) : 256);
    hipLaunchKernelGGL(table_insert_many_kernel, dim3(blocks, n), dim3(256), 0, s, ents, bg ? 0 : 1);
    return hipGetLastError();
}

__global__ void chain_flags_many_kernel(const FlagEnt* __restrict__ ents) {
    const FlagEnt e = ents[blockIdx.y];
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < e.count; k += gridDim.x * blockDim.x) {
        bool eq = e.wsrc[k] == e.wbas[k];
        for (uint32_t j = 0; j < e.dl; ++j) eq &= e.ssrc[(size_t)k * e.dl + j] == e.sbas[(size_t)k * e.dl + j];
        e.flags[k] = eq ? 1 : 0;
    }
}

hipError_t launch_chain_flags_many(const FlagEnt* ents, uint32_t n, uint32_t max_count, hipStream_t s) {
    if (n == 0 || max_count == 0) return hipSuccess;
    const uint32_t blocks = std::min<uint32_t>((max_count + 255) / 256, 256);
    hipLaunchKernelGGL(chain_flags_many_kernel, dim3(blocks, n), dim3(256), 0, s, ents);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// splitmix64 counter stream.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_words_kernel(uint64_t* __restrict__ out, int64_t nwords, uint64_t key, int64_t word0) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = splitmix_mix(key + (uint64_t)(word0 + i + 1) * 0x9E3779B97F4A7C15ull);
}

__global__ void fill_bytes_kernel(uint8_t* __restrict__ out, int64_t n, uint64_t key, int64_t off) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t pos = (uint64_t)(off + i);
        out[i] = (uint8_t)(splitmix_mix(key + (pos / 8 + 1) * 0x9E3779B97F4A7C15ull) >> (8 * (pos % 8)));
    }
}

hipError_t launch_fill_splitmix(uint8_t* d_out, int64_t n, uint64_t key, int64_t byte_offset, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (byte_offset % 8 == 0 && reinterpret_cast<uintptr_t>(d_out) % 8 == 0) {
        const int64_t nw = n / 8;
        if (nw > 0)
            hipLaunchKernelGGL(fill_words_kernel, dim3(4096), dim3(256), 0, s, reinterpret_cast<uint64_t*>(d_out), nw,
                               key, byte_offset / 8);
        const int64_t done = nw * 8;
        if (done < n)
            hipLaunchKernelGGL(fill_bytes_kernel, dim3(1), dim3(64), 0, s, d_out + done, n - done, key,
                               byte_offset + done);
    } else {
        hipLaunchKernelGGL(fill_bytes_kernel, dim3(4096), dim3(256), 0, s, d_out, n, key, byte_offset);
    }
    return hipGetLastError();
}

}  // namespace rsh
