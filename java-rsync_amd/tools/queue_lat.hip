// queue_lat.hip -- how long the device and the host take between two kernels in the patterns the single-file scan
// uses (developer tool; run under rocprofv3 --kernel-trace and read the gaps between the `busy` and `tiny` kernels).
//
// Each case launches `busy` (~400 us of VALU on one workgroup per CU) and then `tiny`, tagged with the case number,
// so the trace shows the idle gap between them:
//   1  same stream, back to back
//   2  same stream, a hipEventRecord (timing disabled) in between
//   3  same stream, a hipEventRecord (timing) in between
//   4  busy through hipExtLaunchKernelGGL with start/stop events, then tiny
//   5  busy on stream 1, event, stream 2 waits, tiny on stream 2 (cross-queue hand-off)
//   6  busy, event, host hipEventSynchronize, then tiny launched by the host (blocking wake-up)
//   7  busy, event, host spins on hipEventQuery, then tiny launched by the host
//   8  busy, a D2H hipMemcpyAsync of 128 KiB into pinned memory, tiny
//   9  busy, tiny writes 128 KiB straight into pinned host memory, then another tiny
//  10  busy, hipStreamWaitEvent on an event that completed long ago, tiny
//  11  busy through hipExtLaunchKernelGGL with a start event only, then tiny
//  12  busy through hipExtLaunchKernelGGL with a stop event only, then tiny
//  13  busy, then a 128 KiB D2H hipMemcpyAsync into pinned memory: the host time the call itself takes (printed)
//  14  busy on stream 1, event, stream 2 waits, a 128 KiB D2H on stream 2: the host time of the copy call (printed)
//  15  busy, then on stream 2 two 512 KiB D2H hipMemcpyAsync into pinned memory, an event, hipEventSynchronize on it
//      (the single-file scan's table download: under rocprofv3 --memory-copy-trace, are their completions delivered)
//  16  the same with 128 KiB copies
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void busy(float* out, int iters, int tag) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = a * b + 1e-7f;
    if (a == 12345.f) out[blockIdx.x] = a + tag;  // never true: keeps the loop
}
__global__ void tiny(float* out, int tag) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)tag;
}
__global__ void tiny_host(unsigned char* h, int n, int tag) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) h[i] = (unsigned char)tag;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int iters = argc > 2 ? atoi(argv[2]) : 200000;
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    float* d;
    CK(hipMalloc(&d, 4096 * sizeof(float)));
    unsigned char *hp, *dp;
    CK(hipHostMalloc(&hp, 1 << 20, hipHostMallocDefault));
    CK(hipMalloc(&dp, 1 << 20));
    hipEvent_t en, et, ea, eb, old;
    CK(hipEventCreateWithFlags(&en, hipEventDisableTiming));
    CK(hipEventCreate(&et));
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    CK(hipEventCreateWithFlags(&old, hipEventDisableTiming));
    CK(hipEventRecord(old, s1));
    CK(hipStreamSynchronize(s1));
    const dim3 G(256), T(64);
    for (int r = 0; r < reps; ++r) {
        for (int c = 1; c <= 16; ++c) {
            const auto t0 = std::chrono::steady_clock::now();
            double call_us = -1;
            if (c == 4) {
                hipExtLaunchKernelGGL(busy, G, T, 0, s1, ea, eb, 0, d, iters, c);
            } else if (c == 11) {
                hipExtLaunchKernelGGL(busy, G, T, 0, s1, ea, nullptr, 0, d, iters, c);
            } else if (c == 12) {
                hipExtLaunchKernelGGL(busy, G, T, 0, s1, nullptr, eb, 0, d, iters, c);
            } else {
                hipLaunchKernelGGL(busy, G, T, 0, s1, d, iters, c);
            }
            hipStream_t ts = s1;
            switch (c) {
                case 2: CK(hipEventRecord(en, s1)); break;
                case 3: CK(hipEventRecord(et, s1)); break;
                case 5:
                    CK(hipEventRecord(en, s1));
                    CK(hipStreamWaitEvent(s2, en, 0));
                    ts = s2;
                    break;
                case 6:
                    CK(hipEventRecord(en, s1));
                    CK(hipEventSynchronize(en));
                    break;
                case 7:
                    CK(hipEventRecord(en, s1));
                    while (hipEventQuery(en) == hipErrorNotReady) {
                    }
                    break;
                case 8: CK(hipMemcpyAsync(hp, dp, 1 << 17, hipMemcpyDeviceToHost, s1)); break;
                case 9: hipLaunchKernelGGL(tiny_host, dim3(32), dim3(256), 0, s1, hp, 1 << 17, c); break;
                case 10: CK(hipStreamWaitEvent(s1, old, 0)); break;
                case 13: {
                    const auto c0 = std::chrono::steady_clock::now();
                    CK(hipMemcpyAsync(hp, dp, 1 << 17, hipMemcpyDeviceToHost, s1));
                    call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
                    break;
                }
                case 14: {
                    CK(hipEventRecord(en, s1));
                    const auto c0 = std::chrono::steady_clock::now();
                    CK(hipStreamWaitEvent(s2, en, 0));
                    CK(hipMemcpyAsync(hp, dp, 1 << 17, hipMemcpyDeviceToHost, s2));
                    call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
                    break;
                }
                case 15:
                case 16: {
                    const size_t sz = c == 15 ? (1u << 19) : (1u << 17);
                    CK(hipMemcpyAsync(hp, dp, sz, hipMemcpyDeviceToHost, s2));
                    CK(hipMemcpyAsync(hp + sz, dp + sz, sz, hipMemcpyDeviceToHost, s2));
                    CK(hipEventRecord(en, s2));
                    CK(hipEventSynchronize(en));
                    break;
                }
                default: break;
            }
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, ts, d, c);
            CK(hipStreamSynchronize(s1));
            CK(hipStreamSynchronize(s2));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (c == 4) {
                float k = 0;
                CK(hipEventElapsedTime(&k, ea, eb));
                printf("rep %d case %d host %.3f ms (busy by ext events %.3f ms)\n", r, c, ms, k);
            } else if (call_us >= 0) {
                printf("rep %d case %d host %.3f ms (the copy call took %.1f us)\n", r, c, ms, call_us);
            } else {
                printf("rep %d case %d host %.3f ms\n", r, c, ms);
            }
        }
    }
    return 0;
}
