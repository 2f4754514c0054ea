// device_common.h -- __device__ helpers shared by the gfx950 translation units (device.hip: the K1 kernels;
// device_scan.hip: probes and the chain walk; device_io.hip: copies, gathers, the stamped launches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsh {

__device__ __forceinline__ int32_t sbyte(uint8_t v) { return (int32_t)(int8_t)v; }

__device__ __forceinline__ uint32_t slot_hash(uint32_t key) {
    uint32_t h = key * 0x9E3779B1u;
    return h ^ (h >> 15);
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

}  // namespace rsh
