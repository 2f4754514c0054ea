// op_rate.hip -- microbenchmark: issue cost of single VALU instructions on gfx950 (candidates for the MD5 step's
// rotate and adds), by waves per SIMD, independent (8 interleaved chains) and dependent (one chain).
// Output: cycles per instruction per wave (s_memtime, median wave) and SIMD cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

#define OP8(INS)                                                                                       \
    asm volatile(INS(0) "\n\t" INS(1) "\n\t" INS(2) "\n\t" INS(3) "\n\t" INS(4) "\n\t" INS(5) "\n\t" INS(6) \
                 "\n\t" INS(7)                                                                         \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), \
                   "+v"(r[7])                                                                          \
                 : "v"(x), "v"(y))
#define DEP8(INS) \
    asm volatile(INS(0) "\n\t" INS(0) "\n\t" INS(0) "\n\t" INS(0) "\n\t" INS(0) "\n\t" INS(0) "\n\t" INS(0) \
                 "\n\t" INS(0)                                                                         \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), \
                   "+v"(r[7])                                                                          \
                 : "v"(x), "v"(y))

#define I_ADD(k) "v_add_u32 %" #k ", %" #k ", %8"
#define I_ADDLIT(k) "v_add_u32 %" #k ", 0x12345678, %" #k
#define I_ADD3(k) "v_add3_u32 %" #k ", %" #k ", %8, %9"
#define I_ALIGNBIT(k) "v_alignbit_b32 %" #k ", %" #k ", %" #k ", 25"
#define I_BITOP3(k) "v_bitop3_b32 %" #k ", %" #k ", %8, %9 bitop3:0xca"
#define I_LSHLADD(k) "v_lshl_add_u32 %" #k ", %" #k ", 7, %8"
#define I_LSHLOR(k) "v_lshl_or_b32 %" #k ", %" #k ", 7, %8"
#define I_ADDLSHL(k) "v_add_lshl_u32 %" #k ", %" #k ", %8, 7"
#define I_LSHR(k) "v_lshrrev_b32 %" #k ", 25, %" #k
#define I_XAD(k) "v_xad_u32 %" #k ", %" #k ", %8, %9"
#define I_PERM(k) "v_perm_b32 %" #k ", %" #k ", %8, %9"
#define I_ALIGNBYTE(k) "v_alignbyte_b32 %" #k ", %" #k ", %8, 2"
#define I_OR3(k) "v_or3_b32 %" #k ", %" #k ", %8, %9"
#define I_PKADD16(k) "v_pk_add_u16 %" #k ", %" #k ", %8"
#define I_BFI(k) "v_bfi_b32 %" #k ", %" #k ", %8, %9"
#define I_MAD24(k) "v_mad_u32_u24 %" #k ", %" #k ", %8, %9"
#define I_LSHL64(k) "v_lshlrev_b32 %" #k ", 7, %" #k

template <int OP, bool DEP, bool HALF = false>
__global__ __launch_bounds__(256) void op_kernel(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) {
    const int lane = threadIdx.x & 63;
    if (HALF && lane >= 32) iters = 0;  // upper half of every wave idle (exec-masked)
    uint32_t r[8];
    for (int k = 0; k < 8; ++k) r[k] = seed + threadIdx.x * 8 + k;
    const uint32_t x = seed * 3 + lane, y = seed ^ 0x5a5a5a5au;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#define RUN(NAME)          \
    if constexpr (DEP)     \
        DEP8(NAME);        \
    else                   \
        OP8(NAME);
            if constexpr (OP == 0) { RUN(I_ADD) }
            else if constexpr (OP == 1) { RUN(I_ADDLIT) }
            else if constexpr (OP == 2) { RUN(I_ADD3) }
            else if constexpr (OP == 3) { RUN(I_ALIGNBIT) }
            else if constexpr (OP == 4) { RUN(I_BITOP3) }
            else if constexpr (OP == 5) { RUN(I_LSHLADD) }
            else if constexpr (OP == 6) { RUN(I_LSHLOR) }
            else if constexpr (OP == 7) { RUN(I_ADDLSHL) }
            else if constexpr (OP == 8) { RUN(I_LSHR) }
            else if constexpr (OP == 9) { RUN(I_XAD) }
            else if constexpr (OP == 10) { RUN(I_PERM) }
            else if constexpr (OP == 11) { RUN(I_ALIGNBYTE) }
            else if constexpr (OP == 12) { RUN(I_OR3) }
            else if constexpr (OP == 13) { RUN(I_PKADD16) }
            else if constexpr (OP == 14) { RUN(I_BFI) }
            else if constexpr (OP == 15) { RUN(I_MAD24) }
            else { RUN(I_LSHL64) }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
    for (int k = 0; k < 8; ++k) acc ^= r[k];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

static const char* kNames[] = {"v_add_u32", "v_add_u32 lit", "v_add3_u32", "v_alignbit_b32", "v_bitop3_b32",
                               "v_lshl_add_u32", "v_lshl_or_b32", "v_add_lshl_u32", "v_lshrrev_b32", "v_xad_u32",
                               "v_perm_b32", "v_alignbyte_b32", "v_or3_b32", "v_pk_add_u16", "v_bfi_b32",
                               "v_mad_u32_u24", "v_lshlrev_b32"};

template <int OP, bool DEP, bool HALF = false>
void run(int wps) {
    const int blocks = 256 * wps;  // 4 waves per block: one per SIMD -> wps waves per SIMD
    const int iters = 2048;
    uint32_t* out;
    uint64_t* cyc;
    (void)hipMalloc(&out, blocks * 256 * 4);
    (void)hipMalloc(&cyc, blocks * 4 * 8);
    hipLaunchKernelGGL((op_kernel<OP, DEP, HALF>), dim3(blocks), dim3(256), 0, 0, out, cyc, 16, 1u);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL((op_kernel<OP, DEP, HALF>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1u);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h(blocks * 4);
    (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double ins = (double)iters * 4 * 8;
    const double med = (double)h[h.size() / 2];
    printf("%-16s %s%s waves/SIMD=%d: %6.2f cyc/instr/wave   SIMD cyc per wave-instr %5.2f\n", kNames[OP],
           DEP ? "dep  " : "indep", HALF ? " half-exec" : "", wps, med / ins, med / ins / wps);
    fflush(stdout);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

template <int OP>
void all() {
    for (int w : {1, 2, 4}) run<OP, false>(w);
    run<OP, true>(1);
    run<OP, true>(2);
}

int main() {
    for (int w : {1, 2, 4}) run<0, false, true>(w);
    for (int w : {1, 2, 4}) run<3, false, true>(w);
    all<0>(); all<3>(); all<4>();
    return 0;
}
