// mfma_layout -- developer check of the v_mfma_i32_16x16x64_i8 operand / accumulator lane maps assumed
// by the MFMA weak-sum path: lane l holds A[l&15][16(l>>4)+j] and B[16(l>>4)+j][l&15] (j = byte 0..15),
// C/D reg r of lane l is C[4(l>>4)+r][l&15].  Exits 0 iff the product matches a CPU matmul.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const v4i* a, const v4i* b, v4i* c) {
    const int l = threadIdx.x;
    v4i acc = {0, 0, 0, 0};
    c[l] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
}

int main() {
    signed char A[16][64], Bm[64][16];
    srand(7);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 64; ++j) A[i][j] = (signed char)(rand() % 256 - 128);
    for (int i = 0; i < 64; ++i)
        for (int j = 0; j < 16; ++j) Bm[i][j] = (signed char)(rand() % 256 - 128);
    signed char fa[64][16], fb[64][16];
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 16; ++j) {
            fa[l][j] = A[l & 15][16 * (l >> 4) + j];
            fb[l][j] = Bm[16 * (l >> 4) + j][l & 15];
        }
    v4i *da, *db, *dc;
    hipMalloc(&da, 64 * 16);
    hipMalloc(&db, 64 * 16);
    hipMalloc(&dc, 64 * 16);
    hipMemcpy(da, fa, 1024, hipMemcpyHostToDevice);
    hipMemcpy(db, fb, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc);
    int hc[64][4];
    hipMemcpy(hc, dc, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * (l >> 4) + r, col = l & 15;
            int ref = 0;
            for (int kk = 0; kk < 64; ++kk) ref += A[row][kk] * Bm[kk][col];
            if (ref != hc[l][r]) ++bad;
        }
    printf("mfma_i32_16x16x64_i8 layout: %s (%d mismatches)\n", bad ? "MISMATCH" : "ok", bad);
    return bad ? 1 : 0;
}
