// device.hip -- gfx950 (CDNA4) kernels for java-rsync's delta-transfer checksum path.
//
// Integer/byte work, HBM-bound: no MFMA.  Layout in HBM: the file is one flat byte array (caller's
// buffer, 256-B aligned from hipMalloc); per-chunk outputs are struct-of-arrays (weak int32[C],
// strong uint8[C*dl]).  See DESIGN.md for the roofline of each kernel.
#include <hip/hip_runtime.h>

#include "device.h"
#include "md5_core.h"

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

template <int ALIGN>
__device__ __forceinline__ void load_block(const uint8_t* p, uint4 (&q)[4]) {
    if constexpr (ALIGN == 16) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* v = reinterpret_cast<const u32x4*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4 t = __builtin_nontemporal_load(v + i);
            q[i] = make_uint4(t.x, t.y, t.z, t.w);
        }
    } else if constexpr (ALIGN == 4) {
        const uint32_t* v = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
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
template <int ALIGN, int PF>
__global__ __launch_bounds__(64) void block_sums_kernel(const uint8_t* __restrict__ data, int64_t n, uint32_t B,
                                                        uint32_t nchunks, uint32_t dl, uint32_t seed,
                                                        int32_t* __restrict__ weak_out,
                                                        uint8_t* __restrict__ strong_out) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
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
        if ((uint32_t)j < nfull) load_block<ALIGN>(p + 64 * j, q[j]);

    uint32_t i = 0;
    // Steady state: every consumed slot is refilled PF blocks ahead, unconditionally.
    for (; i + 2 * PF <= nfull; i += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            uint32_t m[16];
            unpack(q[j], m);
            load_block<ALIGN>(p + 64 * (size_t)(i + j + PF), q[j]);
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
                if (blk + PF < nfull) load_block<ALIGN>(p + 64 * (size_t)(blk + PF), q[j]);
                weak_block(m, s1, u, 64 * blk);
                md5_compress(st, m);
            }
        }
    }
    md5_tail(st, p + 64 * (size_t)nfull, L & 63u, seed, (uint64_t)L + 4, s1, u, 64 * nfull);

    const int32_t s2 = (int32_t)(L * (uint32_t)s1 - (uint32_t)u);
    weak_out[c] = (int32_t)(((uint32_t)s1 & 0xFFFFu) | ((uint32_t)s2 << 16));
    uint8_t* o = strong_out + (size_t)c * dl;
    for (uint32_t k = 0; k < dl; ++k) {
        const uint32_t word = k < 4 ? st.a : k < 8 ? st.b : k < 12 ? st.c : st.d;
        o[k] = (uint8_t)(word >> (8 * (k & 3)));
    }
}

hipError_t launch_block_sums(const uint8_t* d_data, int64_t n, uint32_t B, uint32_t nchunks, uint32_t dl,
                             uint32_t seed_word, int32_t* d_weak, uint8_t* d_strong, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    const dim3 block(64);
    const dim3 grid((nchunks + 63) / 64);
    const uintptr_t addr = reinterpret_cast<uintptr_t>(d_data);
    if ((B % 16) == 0 && (addr % 16) == 0)
        hipLaunchKernelGGL((block_sums_kernel<16, 4>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong);
    else if ((B % 4) == 0 && (addr % 4) == 0)
        hipLaunchKernelGGL((block_sums_kernel<4, 2>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong);
    else
        hipLaunchKernelGGL((block_sums_kernel<1, 1>), grid, block, 0, s, d_data, n, B, nchunks, dl, seed_word,
                           d_weak, d_strong);
    return hipGetLastError();
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

__global__ void table_clear_kernel(unsigned long long* slots, uint32_t nslots) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += gridDim.x * blockDim.x) slots[i] = 0ull;
}

__global__ void table_insert_kernel(unsigned long long* slots, uint32_t mask, const int32_t* __restrict__ keys,
                                    uint32_t nkeys) {
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

hipError_t launch_table_clear(unsigned long long* d_slots, uint32_t nslots, hipStream_t s) {
    hipLaunchKernelGGL(table_clear_kernel, dim3(std::min<uint32_t>((nslots + 255) / 256, 2048u)), dim3(256), 0, s,
                       d_slots, nslots);
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
// Probe: first position in [a, b) whose Sender rolling key hits the table.  One workgroup per
// aligned block [kB, kB + B); 256 lanes each own a contiguous segment of positions.  Lane start sums
// come from a workgroup scan of per-segment byte sums of the two streams x[p] and x[p + B] (prefix
// identities in the header comment of device.h), then each lane rolls with the exact Java updates.
// ------------------------------------------------------------------------------------------------
constexpr int PROBE_THREADS = 256;

__device__ __forceinline__ int32_t roll_sub(int32_t cs, int32_t w, int32_t x) {  // Rolling.java:56-60
    const uint32_t lo = ((uint32_t)cs & 0xFFFFu) - (uint32_t)x;
    const uint32_t hi = ((uint32_t)cs >> 16) - (uint32_t)w * (uint32_t)x;
    return (int32_t)((lo & 0xFFFFu) | (hi << 16));
}
__device__ __forceinline__ int32_t roll_add(int32_t cs, int32_t x) {  // Rolling.java:25-29
    const uint32_t lo = ((uint32_t)cs & 0xFFFFu) + (uint32_t)x;
    const uint32_t hi = ((uint32_t)cs >> 16) + lo;
    return (int32_t)((lo & 0xFFFFu) | (hi << 16));
}

__global__ __launch_bounds__(PROBE_THREADS) void probe_first_kernel(ProbeArgs A, int64_t k0) {
    const int64_t k = k0 + blockIdx.x;
    const int64_t o = k * (int64_t)A.B;
    const int64_t n = A.n;
    const int64_t B = A.B;
    const int64_t lo_pos = A.a > o ? A.a : o;
    const int64_t hi_pos = A.b < o + B ? A.b : o + B;
    if (lo_pos >= hi_pos) return;  // uniform over the workgroup

    const int t = threadIdx.x;
    const int64_t seg = (B + PROBE_THREADS - 1) / PROBE_THREADS;
    const int64_t q = o + t * seg;
    const int64_t qend_a = (q + seg < n ? q + seg : n);

    // per-segment sums of stream A: [q, q+seg) and stream B: [q+B, q+B+seg), both clipped at n
    int32_t sa = 0, sa2 = 0, sb = 0, sb2 = 0;
    for (int64_t j = q; j < qend_a; ++j) {
        const int32_t x = sbyte(A.data[j]);
        sa += x;
        sa2 += (int32_t)((uint32_t)(j - o) * (uint32_t)x);
    }
    const int64_t qb = q + B;
    const int64_t qend_b = (qb + seg < n ? qb + seg : n);
    for (int64_t j = qb; j < qend_b; ++j) {
        const int32_t x = sbyte(A.data[j]);
        sb += x;
        sb2 += (int32_t)((uint32_t)(j - o) * (uint32_t)x);
    }
    // exclusive scan over lanes (simple LDS Hillis-Steele; 4 values)
    __shared__ int32_t sh[4][PROBE_THREADS];
    sh[0][t] = sa;
    sh[1][t] = sa2;
    sh[2][t] = sb;
    sh[3][t] = sb2;
    __syncthreads();
    for (int d = 1; d < PROBE_THREADS; d <<= 1) {
        int32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
        if (t >= d) {
            v0 = sh[0][t - d];
            v1 = sh[1][t - d];
            v2 = sh[2][t - d];
            v3 = sh[3][t - d];
        }
        __syncthreads();
        sh[0][t] += v0;
        sh[1][t] += v1;
        sh[2][t] += v2;
        sh[3][t] += v3;
        __syncthreads();
    }
    const int32_t pa = sh[0][t] - sa, pa2 = sh[1][t] - sa2;  // P1'(q), P2'(q)
    const int32_t pb = sh[2][t] - sb, pb2 = sh[3][t] - sb2;  // sums over [o+B, q+B) clipped
    if (q >= hi_pos || q >= n) return;

    // T(o) -> P1'(e0), P2'(e0) with e0 = min(o + B, n)
    const int32_t To = A.aligned_weak[k];
    const int64_t e0 = (o + B < n ? o + B : n);
    const uint32_t s1o = (uint32_t)To & 0xFFFFu;
    const uint32_t s2o = (uint32_t)To >> 16;
    const uint32_t P1e = s1o + (uint32_t)pb;
    const uint32_t P2e = (uint32_t)(e0 - o) * s1o - s2o + (uint32_t)pb2;
    const int64_t endq = (q + B < n ? q + B : n);
    const uint32_t s1 = P1e - (uint32_t)pa;
    const uint32_t s2 = (uint32_t)(endq - o) * s1 - (P2e - (uint32_t)pa2);
    // R(q) = T(q) + E(q)
    const int64_t nb = n - B;
    auto clampB = [&](int64_t p) { return p < nb ? p : nb; };
    const uint32_t ehi = A.e_hi + A.e_lo * (uint32_t)(clampB(q) - clampB(A.anchor));
    int32_t R = (int32_t)(((s1 + A.e_lo) & 0xFFFFu) | ((s2 + ehi) << 16));

    const int64_t pend = (q + seg < hi_pos ? q + seg : hi_pos);
    for (int64_t p = q; p < pend; ++p) {
        if (p >= lo_pos && table_has(A.table, (uint32_t)R)) {
            atomicMin(A.first, (unsigned long long)p);
            return;
        }
        const int64_t w = (n - p < B ? n - p : B);
        R = roll_sub(R, (int32_t)w, sbyte(A.data[p]));
        if (n - (p + 1) >= B) R = roll_add(R, sbyte(A.data[p + B]));
    }
}

hipError_t launch_probe_first(const ProbeArgs& args, hipStream_t s) {
    hipError_t e = hipMemsetAsync(args.first, 0xFF, sizeof(unsigned long long), s);  // "none" = all ones
    if (e != hipSuccess) return e;
    if (args.a >= args.b) return hipSuccess;
    const int64_t k0 = args.a / args.B;
    const int64_t k1 = (args.b - 1) / args.B;
    hipLaunchKernelGGL(probe_first_kernel, dim3((uint32_t)(k1 - k0 + 1)), dim3(PROBE_THREADS), 0, s, args, k0);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// True weak sums at arbitrary positions (one workgroup per position, wave-reduced).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void window_weak_kernel(const uint8_t* __restrict__ data, int64_t n, uint32_t B,
                                                          const int64_t* __restrict__ pos, int32_t* __restrict__ out) {
    const int64_t p = pos[blockIdx.x];
    const int64_t w = (n - p < (int64_t)B ? n - p : (int64_t)B);
    int32_t s1 = 0, u = 0;
    for (int64_t i = threadIdx.x; i < w; i += blockDim.x) {
        const int32_t x = sbyte(data[p + i]);
        s1 += x;
        u += (int32_t)((uint32_t)i * (uint32_t)x);
    }
    __shared__ int32_t r1[256], r2[256];
    r1[threadIdx.x] = s1;
    r2[threadIdx.x] = u;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) {
            r1[threadIdx.x] += r1[threadIdx.x + d];
            r2[threadIdx.x] += r2[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const uint32_t S1 = (uint32_t)r1[0];
        const uint32_t S2 = (uint32_t)w * S1 - (uint32_t)r2[0];
        out[blockIdx.x] = (int32_t)((S1 & 0xFFFFu) | (S2 << 16));
    }
}

hipError_t launch_window_weak(const uint8_t* d_data, int64_t n, uint32_t B, const int64_t* d_pos, uint32_t npos,
                              int32_t* d_out, hipStream_t s) {
    if (npos == 0) return hipSuccess;
    hipLaunchKernelGGL(window_weak_kernel, dim3(npos), dim3(256), 0, s, d_data, n, B, d_pos, d_out);
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
