// device_roll.h -- device helpers shared by the Sender's search kernels (device_scan.hip: the range probes;
// device_chain.hip: the batched scan's chain walk): the probe tile's shape, Rolling's add / subtract
// (Rolling.java:25-60) and 16 source bytes held packed in four VGPRs.
#pragma once
#include <hip/hip_runtime.h>

#include "device.h"

namespace rsh {

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

}  // namespace rsh
