// Which XCD does CU index i of a stream CU mask (hipExtStreamCreateWithCUMask) belong to?  For a few
// single-CU masks, launch 16 workgroups on the masked stream and record HW_REG_XCC_ID of each.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <thread>

__global__ void xcc_kernel(int* out) {
    if (threadIdx.x == 0) {
        unsigned v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        out[blockIdx.x] = (int)(v & 0xF);
    }
}

int main() {
    int* d;
    int h[16];
    (void)hipMalloc(&d, 16 * sizeof(int));
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    printf("CUs %d, host threads %u\n", p.multiProcessorCount, std::thread::hardware_concurrency());
    const int cus[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 16, 31, 32, 33, 40, 64, 96, 128, 255};
    for (int cu : cus) {
        uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        mask[cu / 32] = 1u << (cu % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) { printf("mask create failed\n"); return 1; }
        hipLaunchKernelGGL(xcc_kernel, dim3(16), dim3(64), 0, s, d);
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("cu %3d -> xcc", cu);
        for (int i = 0; i < 16; ++i) printf(" %d", h[i]);
        printf("\n");
        (void)hipStreamDestroy(s);
    }
    return 0;
}
