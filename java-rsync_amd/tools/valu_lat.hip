// valu_lat.hip -- microbenchmark: throughput of MD5-step chains on gfx950 by waves/SIMD, active lanes and
// step formulation.  Question: the K1 MD5 lane chain runs at 2 waves/SIMD (131072 chunks of 128 KiB fill
// 2048 waves); is it bound by the dependent-issue latency of a wave, and which formulation / lane
// layout gets more lane-steps per SIMD cycle?
// Output: lane-steps per SIMD cycle (s_memtime, median wave), for each configuration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

// KIND 0: compiler's form   f = bitop3(b,c,d); t = a + m; t = add3(t, f, K); t = alignbit(t,t,r); a = t + b
// KIND 1: off-path add3     t = add3(a, m, K); f = bitop3(b,c,d); t = t + f; t = alignbit; a = t + b
// KIND 2: literal K         t = m + K(lit); t = t + a; f = bitop3; t = t + f; alignbit; a = t + b
#define STEP0(a, b, c, d, r)                                                                          \
    asm volatile("v_bitop3_b32 %1, %3, %4, %5 bitop3:0xac\n\t"                                        \
                 "v_add_u32 %2, %0, %6\n\t"                                                           \
                 "v_add3_u32 %2, %2, %1, %7\n\t"                                                      \
                 "v_alignbit_b32 %2, %2, %2, " #r "\n\t"                                              \
                 "v_add_u32 %0, %2, %3"                                                               \
                 : "+v"(a), "=&v"(f), "=&v"(t)                                                        \
                 : "v"(b), "v"(c), "v"(d), "v"(m), "s"(K))
#define STEP1(a, b, c, d, r)                                                                          \
    asm volatile("v_add3_u32 %2, %0, %6, %7\n\t"                                                      \
                 "v_bitop3_b32 %1, %3, %4, %5 bitop3:0xac\n\t"                                        \
                 "v_add_u32 %2, %2, %1\n\t"                                                           \
                 "v_alignbit_b32 %2, %2, %2, " #r "\n\t"                                              \
                 "v_add_u32 %0, %2, %3"                                                               \
                 : "+v"(a), "=&v"(f), "=&v"(t)                                                        \
                 : "v"(b), "v"(c), "v"(d), "v"(m), "s"(K))
#define STEP2(a, b, c, d, r)                                                                          \
    asm volatile("v_add_u32 %2, 0x5a827999, %6\n\t"                                                   \
                 "v_add_u32 %2, %2, %0\n\t"                                                           \
                 "v_bitop3_b32 %1, %3, %4, %5 bitop3:0xac\n\t"                                        \
                 "v_add_u32 %2, %2, %1\n\t"                                                           \
                 "v_alignbit_b32 %2, %2, %2, " #r "\n\t"                                              \
                 "v_add_u32 %0, %2, %3"                                                               \
                 : "+v"(a), "=&v"(f), "=&v"(t)                                                        \
                 : "v"(b), "v"(c), "v"(d), "v"(m), "s"(K))

template <int KIND, bool HALF>
__global__ __launch_bounds__(256) void chain_kernel(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) {
    const int lane = threadIdx.x & 63;
    uint32_t a = seed + threadIdx.x, b = a * 3u, c = a ^ 0x1234u, d = a + 99u, m = a * 7u;
    const uint32_t K = seed * 0x9e3779b9u;
    uint32_t f, t;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (!HALF || lane < 32) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (KIND == 0) {
                    STEP0(a, b, c, d, 25); STEP0(d, a, b, c, 20); STEP0(c, d, a, b, 15); STEP0(b, c, d, a, 10);
                } else if constexpr (KIND == 1) {
                    STEP1(a, b, c, d, 25); STEP1(d, a, b, c, 20); STEP1(c, d, a, b, 15); STEP1(b, c, d, a, 10);
                } else {
                    STEP2(a, b, c, d, 25); STEP2(d, a, b, c, 20); STEP2(c, d, a, b, 15); STEP2(b, c, d, a, 10);
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
    if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND, bool HALF>
void run(const char* name, int wps) {
    const int blocks = 256 * wps;
    const int iters = 1024;
    uint32_t* out;
    uint64_t* cyc;
    (void)hipMalloc(&out, blocks * 256 * 4);
    (void)hipMalloc(&cyc, blocks * 4 * 8);
    hipLaunchKernelGGL((chain_kernel<KIND, HALF>), dim3(blocks), dim3(256), 0, 0, out, cyc, 16, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((chain_kernel<KIND, HALF>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(blocks * 4);
    (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double steps = (double)iters * 16;
    const double med = (double)h[h.size() / 2];
    const double lanes = HALF ? 32 : 64;
    // chip-wide lane-steps per second (wall) -> per SIMD per cycle at the median wave's cycle count
    const double chip_lane_steps = steps * lanes * blocks * 4;
    printf("%-8s lanes=%2d waves/SIMD=%d: %6.2f cyc/step/wave (median)  lane-steps/SIMD/cyc %.2f  wall %.3f ms  "
           "chip %.1f Glane-steps/s\n",
           name, (int)lanes, wps, med / steps, lanes * wps * steps / med, ms, chip_lane_steps / (ms * 1e6));
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    for (int w : {1, 2, 3, 4, 6, 8}) {
        run<0, false>("compiler", w);
        run<1, false>("offpath", w);
        run<2, false>("literal", w);
        run<0, true>("compiler", w);
        run<1, true>("offpath", w);
    }
    return 0;
}
