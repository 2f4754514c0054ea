// md5_core.h -- MD5 compression (RFC 1321) and the rsync weak-sum block update, shared by the gfx950
// kernels (one lane = one message) and the host side (whole-file digest, single resolver windows).
//
// The reference's strong checksum is java.security.MessageDigest("MD5") (util/MD5.java:35-41) over
// block || seed4 truncated to the digest length (Generator.java:891-893, Sender.java:1260-1262).
// The weak sum is Rolling.compute (util/Rolling.java:31-46) over signed bytes, CHAR_OFFSET = 0.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RSH_HD __host__ __device__ __forceinline__
#define RSH_UNROLL _Pragma("unroll")
#else
#define RSH_HD static inline
#define RSH_UNROLL _Pragma("GCC unroll 4")
#endif

namespace rsh {

struct Md5State {
    uint32_t a, b, c, d;
};

RSH_HD Md5State md5_init() { return Md5State{0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u}; }

RSH_HD uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

// Round functions in the forms the gfx950 backend turns into one v_bfi_b32 / v_xor3_b32 each.
#define RSH_MD5_F(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define RSH_MD5_G(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define RSH_MD5_H(x, y, z) ((x) ^ (y) ^ (z))
#define RSH_MD5_I(x, y, z) ((y) ^ ((x) | ~(z)))
#define RSH_MD5_STEP(f, a, b, c, d, m, k, s) (a) = (b) + rsh::rotl32((a) + f((b), (c), (d)) + (m) + (k), (s))

#if defined(__HIP_DEVICE_COMPILE__) && defined(__gfx950__)
// Round 3 on gfx950: one v_bitop3_b32 (0x96 = x ^ y ^ z) -- the backend canonicalises every XOR3 form
// to two v_xor_b32.  t = a + m + k is formed off the critical path; only H + t, the rotate and the
// final add depend on the previous step.
__device__ __forceinline__ uint32_t rsh_h_plus(uint32_t t, uint32_t x, uint32_t y, uint32_t z) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %2, %3, %4 bitop3:0x96\n\tv_add_u32_e32 %0, %1, %0"
        : "=&v"(r)
        : "v"(t), "v"(x), "v"(y), "v"(z));
    return r;
}
#define RSH_MD5_STEP3(a, b, c, d, m, k, s) (a) = (b) + rsh::rotl32(rsh_h_plus((a) + (m) + (k), (b), (c), (d)), (s))
#else
#define RSH_MD5_STEP3(a, b, c, d, m, k, s) RSH_MD5_STEP(RSH_MD5_H, a, b, c, d, m, k, s)
#endif

// One 64-byte block; m[0..15] are the little-endian message words.
RSH_HD void md5_compress(Md5State& st, const uint32_t (&m)[16]) {
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[0], 0xd76aa478u, 7);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[2], 0x242070dbu, 17);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[5], 0x4787c62au, 12);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[6], 0xa8304613u, 17);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[7], 0xfd469501u, 22);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[8], 0x698098d8u, 7);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[11], 0x895cd7beu, 22);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[12], 0x6b901122u, 7);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[13], 0xfd987193u, 12);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[14], 0xa679438eu, 17);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[15], 0x49b40821u, 22);

    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[1], 0xf61e2562u, 5);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[6], 0xc040b340u, 9);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[11], 0x265e5a51u, 14);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[5], 0xd62f105du, 5);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[10], 0x02441453u, 9);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[14], 0xc33707d6u, 9);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[8], 0x455a14edu, 20);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[7], 0x676f02d9u, 14);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);

    RSH_MD5_STEP3(a, b, c, d, m[5], 0xfffa3942u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[8], 0x8771f681u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[11], 0x6d9d6122u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[14], 0xfde5380cu, 23);
    RSH_MD5_STEP3(a, b, c, d, m[1], 0xa4beea44u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[4], 0x4bdecfa9u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[7], 0xf6bb4b60u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[10], 0xbebfbc70u, 23);
    RSH_MD5_STEP3(a, b, c, d, m[13], 0x289b7ec6u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[0], 0xeaa127fau, 11);
    RSH_MD5_STEP3(c, d, a, b, m[3], 0xd4ef3085u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[6], 0x04881d05u, 23);
    RSH_MD5_STEP3(a, b, c, d, m[9], 0xd9d4d039u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[12], 0xe6db99e5u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[15], 0x1fa27cf8u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[2], 0xc4ac5665u, 23);

    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[0], 0xf4292244u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[7], 0x432aff97u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[14], 0xab9423a7u, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[5], 0xfc93a039u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[12], 0x655b59c3u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[10], 0xffeff47du, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[1], 0x85845dd1u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[6], 0xa3014314u, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[4], 0xf7537e82u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[11], 0xbd3af235u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[9], 0xeb86d391u, 21);

    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
}

#if defined(__HIP_DEVICE_COMPILE__) && defined(__gfx950__)
// md5_compress for the streaming kernels on gfx950.  Per step, six instructions of which only
// v_alignbit_b32 is half-rate: m + K (VOP2 with a 32-bit literal), + a, F = v_bitop3_b32, + F, rotate,
// + b.  The compiler's own form puts a half-rate v_add3_u32 (a + m, F, K from an SGPR) on the
// dependency chain; at the 2 waves/SIMD a 16 GiB file at B = 128 KiB leaves, that chain, not issue, set
// the pace (tools/valu_lat.hip: 37 vs 29 cycles per step per wave; 29 = 96% of the SIMD's issue
// bandwidth at 2 waves).  Truth tables for (S0, S1, S2) = (b, c, d): F 0xca, G 0xe4, H 0x96, I 0x39.
#define RSH_LSTEP(BOP, a, b, c, d, m, k, s)                                                              \
    do {                                                                                                 \
        uint32_t t_, f_;                                                                                 \
        asm("v_add_u32 %1, %8, %6\n\tv_add_u32 %1, %1, %0\n\tv_bitop3_b32 %2, %3, %4, %5 bitop3:" BOP      \
            "\n\tv_add_u32 %1, %1, %2\n\tv_alignbit_b32 %1, %1, %1, %7\n\tv_add_u32 %0, %1, %3"              \
            : "+v"(a), "=&v"(t_), "=&v"(f_)                                                              \
            : "v"(b), "v"(c), "v"(d), "v"(m), "i"(32 - (s)), "i"((int)(k)));                             \
    } while (0)
__device__ __forceinline__ void md5_compress_lit(Md5State& st, const uint32_t (&m)[16]) {
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    RSH_LSTEP("0xca", a, b, c, d, m[0], 0xd76aa478u, 7);
    RSH_LSTEP("0xca", d, a, b, c, m[1], 0xe8c7b756u, 12);
    RSH_LSTEP("0xca", c, d, a, b, m[2], 0x242070dbu, 17);
    RSH_LSTEP("0xca", b, c, d, a, m[3], 0xc1bdceeeu, 22);
    RSH_LSTEP("0xca", a, b, c, d, m[4], 0xf57c0fafu, 7);
    RSH_LSTEP("0xca", d, a, b, c, m[5], 0x4787c62au, 12);
    RSH_LSTEP("0xca", c, d, a, b, m[6], 0xa8304613u, 17);
    RSH_LSTEP("0xca", b, c, d, a, m[7], 0xfd469501u, 22);
    RSH_LSTEP("0xca", a, b, c, d, m[8], 0x698098d8u, 7);
    RSH_LSTEP("0xca", d, a, b, c, m[9], 0x8b44f7afu, 12);
    RSH_LSTEP("0xca", c, d, a, b, m[10], 0xffff5bb1u, 17);
    RSH_LSTEP("0xca", b, c, d, a, m[11], 0x895cd7beu, 22);
    RSH_LSTEP("0xca", a, b, c, d, m[12], 0x6b901122u, 7);
    RSH_LSTEP("0xca", d, a, b, c, m[13], 0xfd987193u, 12);
    RSH_LSTEP("0xca", c, d, a, b, m[14], 0xa679438eu, 17);
    RSH_LSTEP("0xca", b, c, d, a, m[15], 0x49b40821u, 22);
    RSH_LSTEP("0xe4", a, b, c, d, m[1], 0xf61e2562u, 5);
    RSH_LSTEP("0xe4", d, a, b, c, m[6], 0xc040b340u, 9);
    RSH_LSTEP("0xe4", c, d, a, b, m[11], 0x265e5a51u, 14);
    RSH_LSTEP("0xe4", b, c, d, a, m[0], 0xe9b6c7aau, 20);
    RSH_LSTEP("0xe4", a, b, c, d, m[5], 0xd62f105du, 5);
    RSH_LSTEP("0xe4", d, a, b, c, m[10], 0x02441453u, 9);
    RSH_LSTEP("0xe4", c, d, a, b, m[15], 0xd8a1e681u, 14);
    RSH_LSTEP("0xe4", b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    RSH_LSTEP("0xe4", a, b, c, d, m[9], 0x21e1cde6u, 5);
    RSH_LSTEP("0xe4", d, a, b, c, m[14], 0xc33707d6u, 9);
    RSH_LSTEP("0xe4", c, d, a, b, m[3], 0xf4d50d87u, 14);
    RSH_LSTEP("0xe4", b, c, d, a, m[8], 0x455a14edu, 20);
    RSH_LSTEP("0xe4", a, b, c, d, m[13], 0xa9e3e905u, 5);
    RSH_LSTEP("0xe4", d, a, b, c, m[2], 0xfcefa3f8u, 9);
    RSH_LSTEP("0xe4", c, d, a, b, m[7], 0x676f02d9u, 14);
    RSH_LSTEP("0xe4", b, c, d, a, m[12], 0x8d2a4c8au, 20);
    RSH_LSTEP("0x96", a, b, c, d, m[5], 0xfffa3942u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[8], 0x8771f681u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[11], 0x6d9d6122u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[14], 0xfde5380cu, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[1], 0xa4beea44u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[4], 0x4bdecfa9u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[7], 0xf6bb4b60u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[10], 0xbebfbc70u, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[13], 0x289b7ec6u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[0], 0xeaa127fau, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[3], 0xd4ef3085u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[6], 0x04881d05u, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[9], 0xd9d4d039u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[12], 0xe6db99e5u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[15], 0x1fa27cf8u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[2], 0xc4ac5665u, 23);
    RSH_LSTEP("0x39", a, b, c, d, m[0], 0xf4292244u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[7], 0x432aff97u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[14], 0xab9423a7u, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[5], 0xfc93a039u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[12], 0x655b59c3u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[3], 0x8f0ccc92u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[10], 0xffeff47du, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[1], 0x85845dd1u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[8], 0x6fa87e4fu, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[6], 0xa3014314u, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[13], 0x4e0811a1u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[4], 0xf7537e82u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[11], 0xbd3af235u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[9], 0xeb86d391u, 21);
    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
}
// md5_compress_lit with the block's weak-sum dot products threaded through rounds 1-2 (as md5_compress_weak).
__device__ __forceinline__ void md5_compress_lit_weak(Md5State& st, const uint32_t (&m)[16], int32_t& a_out,
                                                  int32_t& b_out) {
    int32_t wa0 = 0, wa1 = 0, wb0 = 0, wb1 = 0;
#define RSH_LWA(j) ((j) & 1 ? wa1 : wa0) = __builtin_amdgcn_sdot4((int)m[j], 0x01010101, (j) & 1 ? wa1 : wa0, false)
#define RSH_LWB(j)                                                                                            \
    ((j) & 1 ? wb1 : wb0) = __builtin_amdgcn_sdot4(                                                          \
        (int)m[j], (4 * (j)) | ((4 * (j) + 1) << 8) | ((4 * (j) + 2) << 16) | ((4 * (j) + 3) << 24),           \
        (j) & 1 ? wb1 : wb0, false)
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    RSH_LSTEP("0xca", a, b, c, d, m[0], 0xd76aa478u, 7);
    RSH_LWA(0);
    RSH_LSTEP("0xca", d, a, b, c, m[1], 0xe8c7b756u, 12);
    RSH_LWA(1);
    RSH_LSTEP("0xca", c, d, a, b, m[2], 0x242070dbu, 17);
    RSH_LWA(2);
    RSH_LSTEP("0xca", b, c, d, a, m[3], 0xc1bdceeeu, 22);
    RSH_LWA(3);
    RSH_LSTEP("0xca", a, b, c, d, m[4], 0xf57c0fafu, 7);
    RSH_LWA(4);
    RSH_LSTEP("0xca", d, a, b, c, m[5], 0x4787c62au, 12);
    RSH_LWA(5);
    RSH_LSTEP("0xca", c, d, a, b, m[6], 0xa8304613u, 17);
    RSH_LWA(6);
    RSH_LSTEP("0xca", b, c, d, a, m[7], 0xfd469501u, 22);
    RSH_LWA(7);
    RSH_LSTEP("0xca", a, b, c, d, m[8], 0x698098d8u, 7);
    RSH_LWA(8);
    RSH_LSTEP("0xca", d, a, b, c, m[9], 0x8b44f7afu, 12);
    RSH_LWA(9);
    RSH_LSTEP("0xca", c, d, a, b, m[10], 0xffff5bb1u, 17);
    RSH_LWA(10);
    RSH_LSTEP("0xca", b, c, d, a, m[11], 0x895cd7beu, 22);
    RSH_LWA(11);
    RSH_LSTEP("0xca", a, b, c, d, m[12], 0x6b901122u, 7);
    RSH_LWA(12);
    RSH_LSTEP("0xca", d, a, b, c, m[13], 0xfd987193u, 12);
    RSH_LWA(13);
    RSH_LSTEP("0xca", c, d, a, b, m[14], 0xa679438eu, 17);
    RSH_LWA(14);
    RSH_LSTEP("0xca", b, c, d, a, m[15], 0x49b40821u, 22);
    RSH_LWA(15);

    RSH_LSTEP("0xe4", a, b, c, d, m[1], 0xf61e2562u, 5);
    RSH_LWB(0);
    RSH_LSTEP("0xe4", d, a, b, c, m[6], 0xc040b340u, 9);
    RSH_LWB(1);
    RSH_LSTEP("0xe4", c, d, a, b, m[11], 0x265e5a51u, 14);
    RSH_LWB(2);
    RSH_LSTEP("0xe4", b, c, d, a, m[0], 0xe9b6c7aau, 20);
    RSH_LWB(3);
    RSH_LSTEP("0xe4", a, b, c, d, m[5], 0xd62f105du, 5);
    RSH_LWB(4);
    RSH_LSTEP("0xe4", d, a, b, c, m[10], 0x02441453u, 9);
    RSH_LWB(5);
    RSH_LSTEP("0xe4", c, d, a, b, m[15], 0xd8a1e681u, 14);
    RSH_LWB(6);
    RSH_LSTEP("0xe4", b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    RSH_LWB(7);
    RSH_LSTEP("0xe4", a, b, c, d, m[9], 0x21e1cde6u, 5);
    RSH_LWB(8);
    RSH_LSTEP("0xe4", d, a, b, c, m[14], 0xc33707d6u, 9);
    RSH_LWB(9);
    RSH_LSTEP("0xe4", c, d, a, b, m[3], 0xf4d50d87u, 14);
    RSH_LWB(10);
    RSH_LSTEP("0xe4", b, c, d, a, m[8], 0x455a14edu, 20);
    RSH_LWB(11);
    RSH_LSTEP("0xe4", a, b, c, d, m[13], 0xa9e3e905u, 5);
    RSH_LWB(12);
    RSH_LSTEP("0xe4", d, a, b, c, m[2], 0xfcefa3f8u, 9);
    RSH_LWB(13);
    RSH_LSTEP("0xe4", c, d, a, b, m[7], 0x676f02d9u, 14);
    RSH_LWB(14);
    RSH_LSTEP("0xe4", b, c, d, a, m[12], 0x8d2a4c8au, 20);
    RSH_LWB(15);

    RSH_LSTEP("0x96", a, b, c, d, m[5], 0xfffa3942u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[8], 0x8771f681u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[11], 0x6d9d6122u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[14], 0xfde5380cu, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[1], 0xa4beea44u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[4], 0x4bdecfa9u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[7], 0xf6bb4b60u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[10], 0xbebfbc70u, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[13], 0x289b7ec6u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[0], 0xeaa127fau, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[3], 0xd4ef3085u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[6], 0x04881d05u, 23);
    RSH_LSTEP("0x96", a, b, c, d, m[9], 0xd9d4d039u, 4);
    RSH_LSTEP("0x96", d, a, b, c, m[12], 0xe6db99e5u, 11);
    RSH_LSTEP("0x96", c, d, a, b, m[15], 0x1fa27cf8u, 16);
    RSH_LSTEP("0x96", b, c, d, a, m[2], 0xc4ac5665u, 23);

    RSH_LSTEP("0x39", a, b, c, d, m[0], 0xf4292244u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[7], 0x432aff97u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[14], 0xab9423a7u, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[5], 0xfc93a039u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[12], 0x655b59c3u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[3], 0x8f0ccc92u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[10], 0xffeff47du, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[1], 0x85845dd1u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[8], 0x6fa87e4fu, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[6], 0xa3014314u, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[13], 0x4e0811a1u, 21);
    RSH_LSTEP("0x39", a, b, c, d, m[4], 0xf7537e82u, 6);
    RSH_LSTEP("0x39", d, a, b, c, m[11], 0xbd3af235u, 10);
    RSH_LSTEP("0x39", c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    RSH_LSTEP("0x39", b, c, d, a, m[9], 0xeb86d391u, 21);

    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
    a_out = wa0 + wa1;
    b_out = wb0 + wb1;
#undef RSH_LWA
#undef RSH_LWB
}
#undef RSH_LSTEP
#include "md5_asm.inc"
#else
RSH_HD void md5_compress_lit(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_asm(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_lit_weak(Md5State& st, const uint32_t (&m)[16], int32_t& a, int32_t& b) {
    md5_compress(st, m);
    a = b = 0;
}
RSH_HD void md5_compress_rot4(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_rot16(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_rot4n(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_rot16n(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_asm4(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_asm16(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_k3s_8(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_k3s_16(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_k3s_16_nonop(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
RSH_HD void md5_compress_k3s_16_nop2(Md5State& st, const uint32_t (&m)[16]) { md5_compress(st, m); }
#endif

#if defined(__HIP__)
// md5_compress with the block's weak-sum dot products (Rolling.compute, two v_dot4_i32_i8 per word)
// threaded through rounds 1-2, one per step, into four independent accumulators: they fill the issue
// bubbles of the MD5 dependency chain instead of forming two serial 16-deep dot4 chains of their own.
// On return: a_out = sum of the 64 signed bytes, b_out = sum k * x_k (k = 0..63 within the block).
__device__ __forceinline__ void md5_compress_weak(Md5State& st, const uint32_t (&m)[16], int32_t& a_out,
                                                  int32_t& b_out) {
    int32_t wa0 = 0, wa1 = 0, wb0 = 0, wb1 = 0;
#define RSH_WA(j) ((j) & 1 ? wa1 : wa0) = __builtin_amdgcn_sdot4((int)m[j], 0x01010101, (j) & 1 ? wa1 : wa0, false)
#define RSH_WB(j)                                                                                            \
    ((j) & 1 ? wb1 : wb0) = __builtin_amdgcn_sdot4(                                                          \
        (int)m[j], (4 * (j)) | ((4 * (j) + 1) << 8) | ((4 * (j) + 2) << 16) | ((4 * (j) + 3) << 24),           \
        (j) & 1 ? wb1 : wb0, false)
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[0], 0xd76aa478u, 7);
    RSH_WA(0);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
    RSH_WA(1);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[2], 0x242070dbu, 17);
    RSH_WA(2);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    RSH_WA(3);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
    RSH_WA(4);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[5], 0x4787c62au, 12);
    RSH_WA(5);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[6], 0xa8304613u, 17);
    RSH_WA(6);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[7], 0xfd469501u, 22);
    RSH_WA(7);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[8], 0x698098d8u, 7);
    RSH_WA(8);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
    RSH_WA(9);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
    RSH_WA(10);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[11], 0x895cd7beu, 22);
    RSH_WA(11);
    RSH_MD5_STEP(RSH_MD5_F, a, b, c, d, m[12], 0x6b901122u, 7);
    RSH_WA(12);
    RSH_MD5_STEP(RSH_MD5_F, d, a, b, c, m[13], 0xfd987193u, 12);
    RSH_WA(13);
    RSH_MD5_STEP(RSH_MD5_F, c, d, a, b, m[14], 0xa679438eu, 17);
    RSH_WA(14);
    RSH_MD5_STEP(RSH_MD5_F, b, c, d, a, m[15], 0x49b40821u, 22);
    RSH_WA(15);

    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[1], 0xf61e2562u, 5);
    RSH_WB(0);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[6], 0xc040b340u, 9);
    RSH_WB(1);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[11], 0x265e5a51u, 14);
    RSH_WB(2);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    RSH_WB(3);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[5], 0xd62f105du, 5);
    RSH_WB(4);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[10], 0x02441453u, 9);
    RSH_WB(5);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
    RSH_WB(6);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    RSH_WB(7);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
    RSH_WB(8);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[14], 0xc33707d6u, 9);
    RSH_WB(9);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
    RSH_WB(10);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[8], 0x455a14edu, 20);
    RSH_WB(11);
    RSH_MD5_STEP(RSH_MD5_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
    RSH_WB(12);
    RSH_MD5_STEP(RSH_MD5_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    RSH_WB(13);
    RSH_MD5_STEP(RSH_MD5_G, c, d, a, b, m[7], 0x676f02d9u, 14);
    RSH_WB(14);
    RSH_MD5_STEP(RSH_MD5_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);
    RSH_WB(15);

    RSH_MD5_STEP3(a, b, c, d, m[5], 0xfffa3942u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[8], 0x8771f681u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[11], 0x6d9d6122u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[14], 0xfde5380cu, 23);
    RSH_MD5_STEP3(a, b, c, d, m[1], 0xa4beea44u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[4], 0x4bdecfa9u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[7], 0xf6bb4b60u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[10], 0xbebfbc70u, 23);
    RSH_MD5_STEP3(a, b, c, d, m[13], 0x289b7ec6u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[0], 0xeaa127fau, 11);
    RSH_MD5_STEP3(c, d, a, b, m[3], 0xd4ef3085u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[6], 0x04881d05u, 23);
    RSH_MD5_STEP3(a, b, c, d, m[9], 0xd9d4d039u, 4);
    RSH_MD5_STEP3(d, a, b, c, m[12], 0xe6db99e5u, 11);
    RSH_MD5_STEP3(c, d, a, b, m[15], 0x1fa27cf8u, 16);
    RSH_MD5_STEP3(b, c, d, a, m[2], 0xc4ac5665u, 23);

    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[0], 0xf4292244u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[7], 0x432aff97u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[14], 0xab9423a7u, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[5], 0xfc93a039u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[12], 0x655b59c3u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[10], 0xffeff47du, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[1], 0x85845dd1u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[6], 0xa3014314u, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
    RSH_MD5_STEP(RSH_MD5_I, a, b, c, d, m[4], 0xf7537e82u, 6);
    RSH_MD5_STEP(RSH_MD5_I, d, a, b, c, m[11], 0xbd3af235u, 10);
    RSH_MD5_STEP(RSH_MD5_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    RSH_MD5_STEP(RSH_MD5_I, b, c, d, a, m[9], 0xeb86d391u, 21);

    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
    a_out = wa0 + wa1;
    b_out = wb0 + wb1;
#undef RSH_WA
#undef RSH_WB
}
#endif


// Little-endian 16-byte digest from the state.
RSH_HD void md5_digest_bytes(const Md5State& st, uint8_t out[16]) {
    const uint32_t w[4] = {st.a, st.b, st.c, st.d};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

// The first dl bytes of the digest as the Sender keeps them: Arrays.copyOf(digest, dl)
// (Sender.java:1262) zero-pads past the 16 digest bytes when a peer's header asks for dl > 16.
// Every byte index is a compile-time constant: a runtime-indexed word (even a select chain over k) became a private
// array indexed through scratch memory, which put scratch into every K1 (its first launch on a queue then waited for
// the runtime's scratch allocation).
RSH_HD void store_digest(uint8_t* o, const Md5State& st, uint32_t dl) {
    const uint32_t w[4] = {st.a, st.b, st.c, st.d};
    RSH_UNROLL
    for (uint32_t i = 0; i < 4; ++i)
        RSH_UNROLL
        for (uint32_t j = 0; j < 4; ++j)
            if (4 * i + j < dl) o[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
    for (uint32_t k = 16; k < dl; ++k) o[k] = 0;
}

}  // namespace rsh
