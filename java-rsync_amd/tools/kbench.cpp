// kbench -- developer micro-benchmark of the block-sum kernel variants (device.hip) on one GPU.
// Times each variant with hipEvents on its stream and checks every variant's output against
// variant 0 bit for bit.  usage: kbench <MiB> <B> <dl> <reps> <variant>...
// variant 1000: the production abortable launch (the Sender's speculation: abort word never set);
// variant 1001: the production entry launch_block_sums without an abort word (the Generator);
// variant 1002: the batched launch over KBENCH_FILES (128) equal files cut from the buffer (config 4's shape).
// Its parity check holds when per is a multiple of B (then the files' chunks are the buffer's chunks).
// variant 1003: the segmented launch (the Sender's prefix + phase speculation kernel) over the buffer.
// variant 1005: the production batch planner over ragged files (below).
// variant 1010: the pipelined K1 with its weak sums on the VALU (v_dot4) instead of the MFMAs (energy A/B).
// (The rejected K1 forms measured in rounds 1-4 -- the coalesced kernel's MD5 step forms, LDS-DMA stages, 4 waves per
// SIMD, persistent waves, no-LDS loads -- were deleted after their A/Bs; DESIGN.md sec. 4 keeps the numbers.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "device.h"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

// KBENCH_GATHER=<op bytes>: the Receiver's block gather (gather_ops_kernel) A/Bs instead: <MiB> copied from one buffer
// to another as ops of that many bytes (shuffled order, as matched blocks arrive), variants of launch_gather_ops_variant;
// GB/s counts the bytes read and written.
static int gather_main(int argc, char** argv) {
    const int64_t n = (int64_t)atoll(argv[1]) << 20;
    const int64_t op = atoll(getenv("KBENCH_GATHER"));
    const int reps = atoi(argv[4]);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint8_t *src, *dst;
    CK(hipMalloc(&src, n));
    CK(hipMalloc(&dst, n));
    CK(rsh::launch_fill_splitmix(src, n, 0x5EED, 0, s));
    std::vector<rsh::GatherOp> ops;
    for (int64_t o = 0; o < n; o += op) ops.push_back(rsh::GatherOp{src + o, dst + o, std::min(op, n - o)});
    for (size_t i = ops.size(); i > 1; --i) std::swap(ops[i - 1], ops[(i * 2654435761u) % i]);
    rsh::GatherOp* d_ops;
    CK(hipMalloc(&d_ops, ops.size() * sizeof(rsh::GatherOp)));
    CK(hipMemcpy(d_ops, ops.data(), ops.size() * sizeof(rsh::GatherOp), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> a(1024), b(1024);
    for (int k = 5; k < argc; ++k) {
        const int v = atoi(argv[k]);
        CK(hipMemset(dst, 0, n));
        CK(rsh::launch_gather_ops_variant(v, d_ops, (uint32_t)ops.size(), s));
        CK(hipStreamSynchronize(s));
        bool same = true;
        for (int64_t off : {(int64_t)0, n / 3, n - 8192}) {
            CK(hipMemcpy(a.data(), src + off, 8192, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), dst + off, 8192, hipMemcpyDeviceToHost));
            same = same && a == b;
        }
        float best = 1e30f, tot = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, s));
            CK(rsh::launch_gather_ops_variant(v, d_ops, (uint32_t)ops.size(), s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            tot += ms;
        }
        printf("gather variant %d  n=%lld op=%lld  avg %.3f ms  best %.3f ms  %.1f GB/s (read+write; %.3f of 8 TB/s)  copy=%s\n",
               v, (long long)n, (long long)op, tot / reps, best, 2.0 * n / (tot / reps / 1e3) / 1e9,
               2.0 * n / (tot / reps / 1e3) / 8e12, same ? "ok" : "MISMATCH");
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 6 && getenv("KBENCH_GATHER")) return gather_main(argc, argv);
    if (argc < 6) {
        fprintf(stderr, "usage: kbench <MiB> <B> <dl> <reps> <variant>...\n");
        return 2;
    }
    // KBENCH_TRIM=t: t bytes fewer than the MiB count (a short last chunk, a partial last wave)
    const int64_t n = ((int64_t)atoll(argv[1]) << 20) - (getenv("KBENCH_TRIM") ? atoll(getenv("KBENCH_TRIM")) : 0);
    const uint32_t B = (uint32_t)atoi(argv[2]), dl = (uint32_t)atoi(argv[3]);
    const int reps = atoi(argv[4]);
    const uint32_t C = (uint32_t)((n + B - 1) / B);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint8_t* d;
    int32_t *w0, *w;
    uint8_t *s0, *sx;
    // KBENCH_OFFSET=k: the data starts k bytes past a 256-B aligned allocation (unaligned-base A/B)
    const int64_t off = getenv("KBENCH_OFFSET") ? atoll(getenv("KBENCH_OFFSET")) : 0;
    // KBENCH_PREALLOC=k: k buffers of the same size allocated (and filled) first, as the bench's other pairs are
    for (int k = 0; k < (getenv("KBENCH_PREALLOC") ? atoi(getenv("KBENCH_PREALLOC")) : 0); ++k) {
        uint8_t* pre;
        CK(hipMalloc(&pre, n + 64));
        CK(rsh::launch_fill_splitmix(pre, n, 0x1234 + k, 0, s));
    }
    CK(hipMalloc(&d, n + off + 64));
    d += off;
    CK(hipMalloc(&w0, C * 4));
    CK(hipMalloc(&w, C * 4));
    CK(hipMalloc(&s0, (size_t)C * dl + 1));
    CK(hipMalloc(&sx, (size_t)C * dl + 1));
    CK(rsh::launch_fill_splitmix(d, n, 0x5EED5EED00000000ull, 0, s));
    CK(rsh::launch_block_sums_variant(0, d, n, B, C, dl, 0x04030201u, w0, s0, s));
    CK(hipStreamSynchronize(s));
    std::vector<int32_t> hw0(C), hw(C);
    std::vector<uint8_t> hs0((size_t)C * dl), hs((size_t)C * dl);
    CK(hipMemcpy(hw0.data(), w0, C * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs0.data(), s0, (size_t)C * dl, hipMemcpyDeviceToHost));
    int* abort_word;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&abort_word), 256, hipDeviceMallocUncached));
    CK(hipMemset(abort_word, 0, 256));
    // variant 1002: the batched launch (config 4's shape) over the same buffer cut into KBENCH_FILES files
    const int nfiles = getenv("KBENCH_FILES") ? atoi(getenv("KBENCH_FILES")) : 128;
    std::vector<rsh::K1File> kf;
    const int64_t per = n / nfiles;
    for (int f = 0; f < nfiles; ++f) {
        const uint32_t cf = (uint32_t)((per + B - 1) / B), c0 = (uint32_t)((int64_t)f * per / B);
        kf.push_back(rsh::K1File{d + (int64_t)f * per, per, B, dl, cf, w + c0, sx + (size_t)c0 * dl});
    }
    std::vector<rsh::K1Group> groups;
    std::vector<rsh::K1Lane> lanes;
    int lane_align = 16;
    rsh::plan_block_sums_batch(kf.data(), nfiles, &groups, &lanes, &lane_align);
    rsh::K1Group* d_groups;
    rsh::K1Lane* d_lanes;
    CK(hipMalloc(&d_groups, (groups.size() + 1) * sizeof(rsh::K1Group)));
    CK(hipMalloc(&d_lanes, (lanes.size() + 1) * sizeof(rsh::K1Lane)));
    CK(hipMemcpy(d_groups, groups.data(), groups.size() * sizeof(rsh::K1Group), hipMemcpyHostToDevice));
    if (!lanes.empty()) CK(hipMemcpy(d_lanes, lanes.data(), lanes.size() * sizeof(rsh::K1Lane), hipMemcpyHostToDevice));
    // variant 1005: the production batch planner (plan_block_sums_files, groups expanded on the device) over
    // KBENCH_FILES files of per - KBENCH_RAG bytes each (ragged: every file has a partial last wave and a short
    // chunk); RSH_K1_GATHER picks gathered partial groups or per-lane leftovers.  Parity is not comparable to
    // variant 0 when KBENCH_RAG > 0 (the files' chunk grids differ from the buffer's).
    const int64_t rag = getenv("KBENCH_RAG") ? atoll(getenv("KBENCH_RAG")) : 0;
    std::vector<rsh::K1File> kr;
    for (int f = 0; f < nfiles; ++f) {
        const int64_t len = per - rag;
        const uint32_t c0 = (uint32_t)((int64_t)f * per / B);
        kr.push_back(rsh::K1File{d + (int64_t)f * per, len, B, dl, (uint32_t)((len + B - 1) / B), w + c0,
                                 sx + (size_t)c0 * dl});
    }
    auto launch_rag = [&]() -> hipError_t {
        std::vector<rsh::K1Plan> plans;
        std::vector<rsh::K1Lane> rl;
        int ra = 16;
        bool partial = rsh::tail_gather_on();
        const uint32_t ng = rsh::plan_block_sums_files(kr.data(), nfiles, &plans, &rl, &ra, &partial);
        static rsh::K1Plan* d_plans = nullptr;
        static rsh::K1Group* d_rg = nullptr;
        static rsh::K1Lane* d_rl = nullptr;
        if (!d_plans) {
            CK(hipMalloc(&d_plans, (size_t)(nfiles + 1) * sizeof(rsh::K1Plan)));
            CK(hipMalloc(&d_rg, (size_t)(C / 64 + nfiles + 1) * sizeof(rsh::K1Group)));
            CK(hipMalloc(&d_rl, (size_t)(2 * nfiles + 1) * sizeof(rsh::K1Lane)));
            CK(hipMemcpy(d_plans, plans.data(), plans.size() * sizeof(rsh::K1Plan), hipMemcpyHostToDevice));
            if (!rl.empty()) CK(hipMemcpy(d_rl, rl.data(), rl.size() * sizeof(rsh::K1Lane), hipMemcpyHostToDevice));
            CK(rsh::launch_expand_groups(d_plans, (uint32_t)plans.size(), ng, d_rg, s));
            CK(hipStreamSynchronize(s));
            printf("variant 1005: %u groups (partial %d), %zu lane waves\n", ng, (int)partial, rl.size());
        }
        return rsh::launch_block_sums_batch(d_rg, ng, d_rl, (uint32_t)rl.size(), ra, 0x04030201u, s, nullptr, 0,
                                            partial);
    };
    // variant 1003: the segmented launch (block_sums_seg_kernel) over the whole buffer as one segment; the
    // buffer's base must be such that base - base % 128 is inside the allocation (KBENCH_OFFSET < 128)
    const uint32_t a_off = (uint32_t)(reinterpret_cast<uintptr_t>(d) % 128);
    // KBENCH_SEGTAIL=1: the last full wave's 64 chunks go to the tail list instead (the shift case's tail wave)
    const uint32_t nfull = (uint32_t)(n / B), nw = nfull / 64 - ((getenv("KBENCH_SEGTAIL") && nfull >= 64) ? 1 : 0);
    std::vector<rsh::K1Seg> segs;
    std::vector<rsh::K1Tail> tails;
    int* never;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&never), 256, hipDeviceMallocUncached));
    CK(hipMemset(never, 0, 256));
    for (uint32_t v = 0; v < nw; ++v)
        segs.push_back(rsh::K1Seg{d - a_off + (size_t)v * 64 * B, w + v * 64, sx + (size_t)v * 64 * dl, never, -1, a_off});
    for (uint32_t c = nw * 64; c < C; ++c) tails.push_back(rsh::K1Tail{d, n, w, sx, c});
    rsh::K1Seg* d_segs;
    CK(hipMalloc(&d_segs, segs.size() * sizeof(rsh::K1Seg) + tails.size() * sizeof(rsh::K1Tail) + 64));
    CK(hipMemcpy(d_segs, segs.data(), segs.size() * sizeof(rsh::K1Seg), hipMemcpyHostToDevice));
    rsh::K1Tail* d_tails = reinterpret_cast<rsh::K1Tail*>(d_segs + segs.size());
    if (!tails.empty()) CK(hipMemcpy(d_tails, tails.data(), tails.size() * sizeof(rsh::K1Tail), hipMemcpyHostToDevice));
    auto launch = [&](int v) {
        if (v == 1003)
            return rsh::launch_block_sums_segments(d_segs, (uint32_t)segs.size(), d_tails, (uint32_t)tails.size(),
                                                   (uint32_t)std::count_if(tails.begin(), tails.end(),
                                                                           [&](const rsh::K1Tail& t) {
                                                                               return (int64_t)(t.c + 1) * B <= t.n;
                                                                           }),
                                                   B, dl, 0x04030201u, s);
        if (v == 1005) return launch_rag();
        if (v == 1002)
            return rsh::launch_block_sums_batch(d_groups, (uint32_t)groups.size(), d_lanes, (uint32_t)lanes.size(),
                                                lane_align, 0x04030201u, s);
        if (v == 1000) return rsh::launch_block_sums_variant(-1, d, n, B, C, dl, 0x04030201u, w, sx, s, abort_word, 1);
        if (v == 1010) return rsh::launch_block_sums_variant(1010, d, n, B, C, dl, 0x04030201u, w, sx, s, abort_word, 1);
        if (v == 1001) return rsh::launch_block_sums(d, n, B, C, dl, 0x04030201u, w, sx, s);  // the production entry
        return rsh::launch_block_sums_variant(v, d, n, B, C, dl, 0x04030201u, w, sx, s);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int a = 5; a < argc; ++a) {
        const int v = atoi(argv[a]);
        CK(hipMemset(w, 0, C * 4));
        CK(launch(v));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(hw.data(), w, C * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hs.data(), sx, (size_t)C * dl, hipMemcpyDeviceToHost));
        const bool same = hw == hw0 && hs == hs0;
        float best = 1e30f, tot = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, s));
            CK(launch(v));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            tot += ms;
        }
        printf("variant %d  n=%lld B=%u C=%u  avg %.3f ms  best %.3f ms  %.1f GB/s  parity=%s\n", v, (long long)n, B, C,
               tot / reps, best, n / (tot / reps / 1e3) / 1e9, same ? "ok" : "MISMATCH");
        fflush(stdout);
    }
    return 0;
}
