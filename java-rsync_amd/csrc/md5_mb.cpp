// md5_mb.cpp -- the whole-file MD5s of a segment's files on the host, several files per core.
//
// The Sender digests every source file whole (Sender.java:1241,1272,1300,1315,1326: one MessageDigest fed the
// file's bytes in order, MD5.java:35-41).  One file is one serial MD5 chain: a core runs it at ~1 GB/s, so a
// 16 GiB source is bound there whatever the device does.  A segment of many files is not:
// their chains are independent, and one core can advance 16 of them at once with AVX-512 (8 with AVX2) -- lane
// l of each vector register holds file l's MD5 state, the message words of the 16 current blocks are loaded and
// transposed so that word w of every lane's block sits in one register, and every MD5 step is the scalar step
// on 16 lanes (v_pternlog for F/G/H/I, vprold for the rotate).  A lane whose file ends takes the next file of
// the queue.  The result is exactly RFC 1321 MD5 per file (the CPU tests compare it with hashlib on files cut
// into pieces of every shape, and with the scalar host MD5).
#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <numeric>
#include <thread>
#include <vector>

#include "host_md5.h"
#include "md5_mb.h"

namespace rsh {
namespace {

// One lane's position in its file: the next 64-byte block is either inside one piece (read in place) or is
// assembled in `tail` (a block straddling two pieces, or the one or two padding blocks at the end).
struct Cursor {
    const rsh_piece* p = nullptr;
    int32_t np = 0, pi = 0;
    int64_t off = 0;        // in piece pi
    uint64_t total = 0, done = 0;
    int tail_blocks = 0;    // padding blocks built in tail (1 or 2)
    int tail_left = 0;      // ... still to run
    bool finishing = false; // the padding blocks are in tail
    alignas(64) uint8_t tail[128];

    void start(const rsh_piece* pieces, int32_t n) {
        p = pieces;
        np = n;
        pi = 0;
        off = 0;
        total = 0;
        for (int32_t i = 0; i < n; ++i) total += (uint64_t)pieces[i].len;
        done = 0;
        tail_blocks = tail_left = 0;
        finishing = false;
        skip_empty();
    }
    void skip_empty() {
        while (pi < np && off >= p[pi].len) {
            ++pi;
            off = 0;
        }
    }
    bool finished() const { return finishing && tail_left == 0; }
    // The next block(s): returns a pointer and how many consecutive 64-byte blocks may be read from it.
    const uint8_t* next(int64_t* count) {
        if (finishing) {
            *count = tail_left;
            return tail + 64 * (tail_blocks - tail_left);
        }
        const uint64_t left = total - done;
        if (left >= 64) {
            const int64_t in_piece = p[pi].len - off;
            if (in_piece >= 64) {
                *count = std::min<int64_t>(in_piece / 64, (int64_t)(left / 64));
                return p[pi].data + off;
            }
            // a block straddling pieces: assemble it
            uint8_t* o = tail;
            int64_t need = 64, o_pi = pi, o_off = off;
            while (need > 0) {
                const int64_t take = std::min<int64_t>(need, p[o_pi].len - o_off);
                memcpy(o, p[o_pi].data + o_off, (size_t)take);
                o += take;
                need -= take;
                o_off += take;
                if (o_off >= p[o_pi].len) {
                    ++o_pi;
                    o_off = 0;
                }
            }
            *count = 1;
            return tail;
        }
        // the last bytes, 0x80, zeros and the bit length: one or two blocks
        memset(tail, 0, sizeof(tail));
        size_t k = 0;
        while (k < left) {
            const int64_t take = std::min<int64_t>((int64_t)(left - k), p[pi].len - off);
            memcpy(tail + k, p[pi].data + off, (size_t)take);
            k += (size_t)take;
            off += take;
            skip_empty();
        }
        tail[k] = 0x80;
        tail_blocks = tail_left = k < 56 ? 1 : 2;
        const uint64_t bits = total * 8;
        for (int i = 0; i < 8; ++i) tail[64 * tail_blocks - 8 + i] = (uint8_t)(bits >> (8 * i));
        finishing = true;
        done = total;
        *count = tail_left;
        return tail;
    }
    // Advance past `k` blocks taken from the pointer next() returned.
    void advance(int64_t k) {
        if (finishing) {
            tail_left -= (int)k;
            return;
        }
        const uint64_t bytes = 64 * (uint64_t)k;
        if (p[pi].len - off >= (int64_t)bytes) {
            off += (int64_t)bytes;
        } else {  // the straddling block
            int64_t need = (int64_t)bytes;
            while (need > 0) {
                const int64_t take = std::min<int64_t>(need, p[pi].len - off);
                off += take;
                need -= take;
                if (off >= p[pi].len && need > 0) {
                    ++pi;
                    off = 0;
                }
            }
        }
        done += bytes;
        skip_empty();
    }
};

#define RSH_MB_K                                                                                                      \
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,         \
        0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,     \
        0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,     \
        0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,     \
        0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,     \
        0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,     \
        0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,     \
        0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u
alignas(64) constexpr uint32_t kK[64] = {RSH_MB_K};
// message word and rotate of step i (RFC 1321 3.4)
constexpr uint8_t kW[64] = {0, 1, 2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 1, 6, 11, 0,  5,  10,
                            15, 4, 9, 14, 3,  8,  13, 2,  7,  12, 5,  8,  11, 14, 1,  4,  7, 10, 13, 0,  3,  6,
                            9,  12, 15, 2, 0, 7,  14, 5,  12, 3,  10, 1,  8,  15, 6,  13, 4, 11, 2,  9};

// ---- AVX-512: 16 lanes ----

#define RSH_MB512_STEP(imm, a, b, c, d, i, s)                                                                        \
    a = _mm512_add_epi32(                                                                                            \
        b, _mm512_rol_epi32(_mm512_add_epi32(_mm512_add_epi32(a, _mm512_add_epi32(m[kW[i]], _mm512_set1_epi32((int)kK[i]))), \
                                             _mm512_ternarylogic_epi32(b, c, d, imm)),                               \
                            s))
#define RSH_MB512_R4(imm, i, s0, s1, s2, s3)  \
    RSH_MB512_STEP(imm, a, b, c, d, i, s0);     \
    RSH_MB512_STEP(imm, d, a, b, c, i + 1, s1); \
    RSH_MB512_STEP(imm, c, d, a, b, i + 2, s2); \
    RSH_MB512_STEP(imm, b, c, d, a, i + 3, s3)

__attribute__((target("avx512f"))) void transpose16(__m512i (&r)[16]) {
    __m512i t[16];
    for (int i = 0; i < 16; i += 2) {
        t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
        t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
    }
    for (int i = 0; i < 16; i += 4) {
        r[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
        r[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
        r[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
        r[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    // r[4q + j] holds, per 128-bit lane k, word (4k + j') of rows 4q..4q+3 (j' = 0, 1, 2, 3 for j = 0, 1, 2, 3)
    for (int j = 0; j < 4; ++j) {
        const __m512i x0 = _mm512_shuffle_i32x4(r[j], r[4 + j], 0x88);   // lanes 0,2 of rows 0-3 / 4-7
        const __m512i x1 = _mm512_shuffle_i32x4(r[j], r[4 + j], 0xDD);   // lanes 1,3
        const __m512i y0 = _mm512_shuffle_i32x4(r[8 + j], r[12 + j], 0x88);
        const __m512i y1 = _mm512_shuffle_i32x4(r[8 + j], r[12 + j], 0xDD);
        t[j] = _mm512_shuffle_i32x4(x0, y0, 0x88);       // word j      (128-bit lane 0 of every row group)
        t[8 + j] = _mm512_shuffle_i32x4(x0, y0, 0xDD);   // word 8 + j
        t[4 + j] = _mm512_shuffle_i32x4(x1, y1, 0x88);   // word 4 + j
        t[12 + j] = _mm512_shuffle_i32x4(x1, y1, 0xDD);  // word 12 + j
    }
    for (int i = 0; i < 16; ++i) r[i] = t[i];
}

// `nblocks` blocks of every lane: lane l reads block j at ptr[l] + j * stride[l] (stride 0 for an idle lane).
__attribute__((target("avx512f"))) void blocks16(uint32_t* st, const uint8_t* const* ptr, const int64_t* stride,
                                                 int64_t nblocks) {
    __m512i A = _mm512_loadu_si512(st), B = _mm512_loadu_si512(st + 16), C = _mm512_loadu_si512(st + 32),
            D = _mm512_loadu_si512(st + 48);
    for (int64_t j = 0; j < nblocks; ++j) {
        __m512i m[16];
        for (int l = 0; l < 16; ++l) m[l] = _mm512_loadu_si512(ptr[l] + j * stride[l]);
        transpose16(m);
        __m512i a = A, b = B, c = C, d = D;
        RSH_MB512_R4(0xCA, 0, 7, 12, 17, 22);
        RSH_MB512_R4(0xCA, 4, 7, 12, 17, 22);
        RSH_MB512_R4(0xCA, 8, 7, 12, 17, 22);
        RSH_MB512_R4(0xCA, 12, 7, 12, 17, 22);
        RSH_MB512_R4(0xE4, 16, 5, 9, 14, 20);
        RSH_MB512_R4(0xE4, 20, 5, 9, 14, 20);
        RSH_MB512_R4(0xE4, 24, 5, 9, 14, 20);
        RSH_MB512_R4(0xE4, 28, 5, 9, 14, 20);
        RSH_MB512_R4(0x96, 32, 4, 11, 16, 23);
        RSH_MB512_R4(0x96, 36, 4, 11, 16, 23);
        RSH_MB512_R4(0x96, 40, 4, 11, 16, 23);
        RSH_MB512_R4(0x96, 44, 4, 11, 16, 23);
        RSH_MB512_R4(0x39, 48, 6, 10, 15, 21);
        RSH_MB512_R4(0x39, 52, 6, 10, 15, 21);
        RSH_MB512_R4(0x39, 56, 6, 10, 15, 21);
        RSH_MB512_R4(0x39, 60, 6, 10, 15, 21);
        A = _mm512_add_epi32(A, a);
        B = _mm512_add_epi32(B, b);
        C = _mm512_add_epi32(C, c);
        D = _mm512_add_epi32(D, d);
    }
    _mm512_storeu_si512(st, A);
    _mm512_storeu_si512(st + 16, B);
    _mm512_storeu_si512(st + 32, C);
    _mm512_storeu_si512(st + 48, D);
}

// ---- AVX2: 8 lanes ----

__attribute__((target("avx2"))) inline __m256i rol8(__m256i x, int s) {
    return _mm256_or_si256(_mm256_slli_epi32(x, s), _mm256_srli_epi32(x, 32 - s));
}
__attribute__((target("avx2"))) inline __m256i f8(int r, __m256i x, __m256i y, __m256i z) {
    switch (r) {
        case 0: return _mm256_xor_si256(z, _mm256_and_si256(x, _mm256_xor_si256(y, z)));
        case 1: return _mm256_xor_si256(y, _mm256_and_si256(z, _mm256_xor_si256(x, y)));
        case 2: return _mm256_xor_si256(_mm256_xor_si256(x, y), z);
        default: return _mm256_xor_si256(y, _mm256_or_si256(x, _mm256_xor_si256(z, _mm256_set1_epi32(-1))));
    }
}
#define RSH_MB256_STEP(a, b, c, d, i, s)                                                                       \
    a = _mm256_add_epi32(                                                                                      \
        b, rol8(_mm256_add_epi32(_mm256_add_epi32(a, _mm256_add_epi32(m[kW[i]], _mm256_set1_epi32((int)kK[i]))), \
                                 f8((i) >> 4, b, c, d)),                                                       \
                s))

__attribute__((target("avx2"))) void transpose8(__m256i (&r)[8]) {
    __m256i t[8];
    for (int i = 0; i < 8; i += 2) {
        t[i] = _mm256_unpacklo_epi32(r[i], r[i + 1]);
        t[i + 1] = _mm256_unpackhi_epi32(r[i], r[i + 1]);
    }
    __m256i u[8];
    for (int i = 0; i < 8; i += 4) {
        u[i] = _mm256_unpacklo_epi64(t[i], t[i + 2]);
        u[i + 1] = _mm256_unpackhi_epi64(t[i], t[i + 2]);
        u[i + 2] = _mm256_unpacklo_epi64(t[i + 1], t[i + 3]);
        u[i + 3] = _mm256_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    for (int j = 0; j < 4; ++j) {
        r[j] = _mm256_permute2x128_si256(u[j], u[4 + j], 0x20);
        r[4 + j] = _mm256_permute2x128_si256(u[j], u[4 + j], 0x31);
    }
}

__attribute__((target("avx2"))) void blocks8(uint32_t* st, const uint8_t* const* ptr, const int64_t* stride,
                                             int64_t nblocks) {
    __m256i A = _mm256_loadu_si256((const __m256i*)st), B = _mm256_loadu_si256((const __m256i*)(st + 8)),
            C = _mm256_loadu_si256((const __m256i*)(st + 16)), D = _mm256_loadu_si256((const __m256i*)(st + 24));
    for (int64_t j = 0; j < nblocks; ++j) {
        __m256i lo[8], hi[8], m[16];
        for (int l = 0; l < 8; ++l) {
            const uint8_t* q = ptr[l] + j * stride[l];
            lo[l] = _mm256_loadu_si256((const __m256i*)q);
            hi[l] = _mm256_loadu_si256((const __m256i*)(q + 32));
        }
        transpose8(lo);
        transpose8(hi);
        for (int w = 0; w < 8; ++w) {
            m[w] = lo[w];
            m[8 + w] = hi[w];
        }
        __m256i a = A, b = B, c = C, d = D;
        static constexpr int kS[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
        for (int i = 0; i < 64; i += 4) {
            const int* s = kS[i >> 4];
            RSH_MB256_STEP(a, b, c, d, i, s[0]);
            RSH_MB256_STEP(d, a, b, c, i + 1, s[1]);
            RSH_MB256_STEP(c, d, a, b, i + 2, s[2]);
            RSH_MB256_STEP(b, c, d, a, i + 3, s[3]);
        }
        A = _mm256_add_epi32(A, a);
        B = _mm256_add_epi32(B, b);
        C = _mm256_add_epi32(C, c);
        D = _mm256_add_epi32(D, d);
    }
    _mm256_storeu_si256((__m256i*)st, A);
    _mm256_storeu_si256((__m256i*)(st + 8), B);
    _mm256_storeu_si256((__m256i*)(st + 16), C);
    _mm256_storeu_si256((__m256i*)(st + 24), D);
}

using BlocksFn = void (*)(uint32_t*, const uint8_t* const*, const int64_t*, int64_t);

// One thread: up to `lanes` files in flight, the next file of the shared queue into every lane that frees.
void run_lanes(const Md5File* files, const int32_t* order, int32_t nfiles, std::atomic<int32_t>* next,
               uint8_t (*out)[16], int lanes, int width, BlocksFn fn) {
    alignas(64) static thread_local uint8_t zero[64];
    std::vector<Cursor> cur((size_t)width);
    std::vector<int32_t> file((size_t)width, -1);
    alignas(64) uint32_t st[4 * 16];
    const uint8_t* ptr[16];
    int64_t stride[16];
    const Md5State init = md5_init();
    for (;;) {
        int active = 0;
        for (int l = 0; l < width; ++l) {
            if (file[(size_t)l] < 0 && l < lanes) {
                const int32_t k = next->fetch_add(1, std::memory_order_relaxed);
                if (k < nfiles) {
                    const int32_t f = order[k];
                    file[(size_t)l] = f;
                    cur[(size_t)l].start(files[f].pieces, files[f].npieces);
                    st[l] = init.a;
                    st[width + l] = init.b;
                    st[2 * width + l] = init.c;
                    st[3 * width + l] = init.d;
                }
            }
            active += file[(size_t)l] >= 0;
        }
        if (active == 0) return;
        int64_t burst = INT64_MAX;
        for (int l = 0; l < width; ++l) {
            if (file[(size_t)l] < 0) {
                ptr[l] = zero;
                stride[l] = 0;
                continue;
            }
            Cursor& c = cur[(size_t)l];
            int64_t cnt = 0;
            ptr[l] = c.next(&cnt);
            stride[l] = 64;
            burst = std::min(burst, cnt);
        }
        burst = std::min<int64_t>(burst, 1 << 14);  // bounded bursts: a lane whose file ends soon is refilled soon
        fn(st, ptr, stride, burst);
        for (int l = 0; l < width; ++l) {
            if (file[(size_t)l] < 0) continue;
            Cursor& c = cur[(size_t)l];
            c.advance(burst);
            if (c.finished()) {
                const Md5State s{st[l], st[width + l], st[2 * width + l], st[3 * width + l]};
                md5_digest_bytes(s, out[file[(size_t)l]]);
                file[(size_t)l] = -1;
            }
        }
    }
}

void scalar_file(const Md5File& f, uint8_t out[16]) {
    HostMd5 m;
    for (int32_t i = 0; i < f.npieces; ++i)
        if (f.pieces[i].len > 0) m.update(f.pieces[i].data, (size_t)f.pieces[i].len);
    m.final(out);
}

}  // namespace

int md5_simd_width() {
    static const int w = [] {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx512f")) return 16;
        if (__builtin_cpu_supports("avx2")) return 8;
        return 1;
    }();
    return w;
}

void md5_files(const Md5File* files, int32_t nfiles, uint8_t (*out)[16], int threads, int force_width) {
    if (nfiles <= 0) return;
    const int width = force_width > 0 ? std::min(force_width, md5_simd_width()) : md5_simd_width();
    threads = std::max(1, std::min(threads, nfiles));
    if (width == 1 || nfiles == 1) {  // one chain per file: the scalar MD5 on a thread each
        std::atomic<int32_t> next{0};
        auto work = [&] {
            for (int32_t k; (k = next.fetch_add(1)) < nfiles;) scalar_file(files[k], out[k]);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < threads; ++t) th.emplace_back(work);
        work();
        for (std::thread& t : th) t.join();
        return;
    }
    // largest files first (the chains run at one rate: the longest one sets the end)
    std::vector<uint64_t> size((size_t)nfiles, 0);
    for (int32_t f = 0; f < nfiles; ++f)
        for (int32_t i = 0; i < files[f].npieces; ++i) size[(size_t)f] += (uint64_t)files[f].pieces[i].len;
    std::vector<int32_t> order((size_t)nfiles);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return size[(size_t)x] > size[(size_t)y]; });
    // spread the files over the threads first, then over each thread's lanes
    const int lanes = std::min(width, (nfiles + threads - 1) / threads);
    threads = std::min(threads, (nfiles + lanes - 1) / lanes);
    std::atomic<int32_t> next{0};
    const BlocksFn fn = width == 16 ? blocks16 : blocks8;
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t)
        th.emplace_back(run_lanes, files, order.data(), nfiles, &next, out, lanes, width, fn);
    run_lanes(files, order.data(), nfiles, &next, out, lanes, width, fn);
    for (std::thread& t : th) t.join();
}

}  // namespace rsh
