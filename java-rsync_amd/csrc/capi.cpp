// capi.cpp -- the C-ABI of include/rsync_hip.h: contexts, sizing and headers, the single-file Generator and Sender
// entry points (the glue that mirrors Generator.sendItemizeAndChecksums / Sender.sendFiles per-file handling; the
// scan itself is scan.cpp), channel bytes, device memory and the diagnostics ABI.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "device.h"
#include "host_md5.h"
#include "resolver.h"
#include "rsync_hip.h"

#include "ctx.h"
#include "options.h"
#include "rsync_hip_debug.h"

namespace {
// rsh_ctx_create, after ctx_warm: one device-resident Generator + Sender pass of each kind over a small synthetic pair --
// a 50%-modified 8 MiB file at B = 131072 (config 5's shape: the tentative launch and its stop, the poisoned scan's
// flush chain) and a segment of two 50%-modified 1 MiB files at B = 8192 (config 4's: the chain walks, an early
// resolution, the events' copies) -- so that a context's first real call finds every path it takes run once: the
// kernels' first dispatches, the runtime's paths and the library's own code.  A few milliseconds.
int warm_calls(rsh_ctx* c) {
    const uint8_t seed[4] = {1, 2, 3, 4};
    constexpr int64_t n5 = 8 << 20, B5 = 131072, n4 = 1 << 20, B4 = 8192;
    const int64_t bytes = 2 * n5 + 4 * n4;
    void* d = nullptr;
    if (hipMalloc(&d, (size_t)bytes + 4096) != hipSuccess) return RSH_E_DEVICE;
    uint8_t* src5 = static_cast<uint8_t*>(d);
    uint8_t* bas5 = src5 + n5;
    uint8_t* src4 = bas5 + n5;  // two files, then their two bases
    uint8_t* bas4 = src4 + 2 * n4;
    int rc = RSH_OK;
    auto fill_pair = [&](uint8_t* src, uint8_t* bas, int64_t n, int64_t B, uint64_t key) {
        // the basis keeps the source's even blocks and takes its odd ones from another stream
        if (rc == RSH_OK && (rsh_fill_splitmix_device(c, src, n, key, 0) != RSH_OK ||
                             rsh_fill_splitmix_device(c, bas, n, key ^ 0xED17, 0) != RSH_OK ||
                             hipMemcpy2DAsync(bas, (size_t)(2 * B), src, (size_t)(2 * B), (size_t)B, (size_t)(n / (2 * B)),
                                              hipMemcpyDeviceToDevice, c->stream) != hipSuccess))
            rc = RSH_E_DEVICE;
    };
    fill_pair(src5, bas5, n5, B5, 0x5EED5EED00000005ull);
    fill_pair(src4, bas4, 2 * n4, B4, 0x5EED5EED00000004ull);
    rsh_header h5{}, h4{};
    if (rc == RSH_OK) rc = rsh_header_make((int32_t)B5, 4, n5, &h5);
    if (rc == RSH_OK) rc = rsh_header_make((int32_t)B4, 3, n4, &h4);
    const int64_t C5 = h5.chunk_count, C4 = h4.chunk_count;
    void* t = nullptr;
    if (rc == RSH_OK && hipMalloc(&t, (size_t)(C5 * 8 + 2 * C4 * 8) + 256) != hipSuccess) rc = RSH_E_DEVICE;
    int32_t* w5 = static_cast<int32_t*>(t);
    uint8_t* s5 = reinterpret_cast<uint8_t*>(w5 + C5);
    int32_t* w4 = reinterpret_cast<int32_t*>(s5 + C5 * 4);
    uint8_t* s4 = reinterpret_cast<uint8_t*>(w4 + 2 * C4);
    std::vector<rsh_event> ev((size_t)(4 * (C5 + C4) + 64));
    int64_t n_ev = 0, lit = 0, mat = 0;
    if (rc == RSH_OK) rc = rsh_block_sums_device(c, bas5, n5, &h5, seed, w5, s5);
    if (rc == RSH_OK)
        rc = rsh_match_scan_device(c, src5, n5, &h5, w5, s5, seed, ev.data(), (int64_t)ev.size(), &n_ev, &lit, &mat,
                                   nullptr);
    if (rc == RSH_OK) {
        rsh_block_job bj[2];
        rsh_scan_job sj[2];
        for (int f = 0; f < 2; ++f) {
            bj[f] = rsh_block_job{bas4 + f * n4, n4, h4, w4 + f * C4, s4 + f * C4 * 3};
            sj[f] = rsh_scan_job{};
            sj[f].d_src = src4 + f * n4;
            sj[f].n = n4;
            sj[f].h = h4;
            sj[f].d_weak = bj[f].d_weak;
            sj[f].d_strong = bj[f].d_strong;
            sj[f].ev = ev.data() + (size_t)f * (ev.size() / 2);
            sj[f].ev_cap = (int64_t)ev.size() / 2;
        }
        rc = rsh_block_sums_batch_device(c, bj, 2, seed);
        if (rc == RSH_OK) rc = rsh_match_scan_batch_device(c, sj, 2, seed, nullptr);
    }
    if (rsh_ctx_sync(c) != RSH_OK && rc == RSH_OK) rc = RSH_E_DEVICE;
    if (t) (void)hipFree(t);
    (void)hipFree(d);
    return rc;
}
}  // namespace

// (ctx.h) the generation wrap: once per ~2^31 launches of a context
int rsh_ctx::next_gen() {
    if (gen >= kGenWrapAt) {
        bool ok = hipDeviceSynchronize() == hipSuccess;  // no launch of this context is running
        ok = ok && hipMemset(abort_word, 0, 256) == hipSuccess;
        ok = ok && rsh::clear_batch_abort_words(batch) == hipSuccess;
        if (ok) gen = 0;  // (a failure leaves the count going: the next call retries)
    }
    return ++gen;
}

extern "C" {

int rsh_abi_version(void) { return RSH_ABI_VERSION; }

const char* rsh_last_error(void) { return g_last_err; }

const char* rsh_strerror(int status) {
    switch (status) {
        case RSH_OK: return "ok";
        case RSH_E_INVAL: return "invalid argument";
        case RSH_E_PROTOCOL: return "checksum header rejected (RsyncProtocolException)";
        case RSH_E_OVERFLOW: return "chunk count is negative or greater than int max (ChunkOverflow)";
        case RSH_E_NOSPACE: return "event buffer too small";
        case RSH_E_DEVICE: return "HIP device error or no gfx950 device";
        case RSH_E_NOMEM: return "out of memory";
        case RSH_E_BUSY: return "context in use by another thread";
        case RSH_E_NOTFOUND: return "file not found (FileViewNotFound)";
        case RSH_E_OPEN: return "file cannot be opened (FileViewOpenFailed)";
        default: return "unknown status";
    }
}

int rsh_device_count(int* count) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (count) *count = c;
    return c > 0 ? RSH_OK : RSH_E_DEVICE;
}

int rsh_ctx_create(int device, rsh_ctx** out) {
    if (!out) return RSH_E_INVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return RSH_E_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RSH_E_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RSH_E_DEVICE;  // kernels are built for gfx950 only
    RSH_HIP(hipSetDevice(device));
    rsh_ctx* c = new (std::nothrow) rsh_ctx();
    if (!c) return RSH_E_NOMEM;
    c->device = device;
    c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->abort_word = nullptr;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->phase, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tab, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_spec, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_phase[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_phase[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_flags, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_prep, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->ev_k1a) != hipSuccess || hipEventCreate(&c->ev_k1b) != hipSuccess ||
        hipEventCreate(&c->ev_gen_a) != hipSuccess || hipEventCreate(&c->ev_gen_b) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rs_tail, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->ev_pha[0]) != hipSuccess || hipEventCreate(&c->ev_phb[0]) != hipSuccess ||
        hipEventCreate(&c->ev_pha[1]) != hipSuccess || hipEventCreate(&c->ev_phb[1]) != hipSuccess ||
        hipExtMallocWithFlags(reinterpret_cast<void**>(&c->abort_word), 256, hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(c->abort_word, 0, 256) != hipSuccess ||  // generations start at 1
        // recorded once, so that a launch may always wait for its buffer set's previous launch
        hipEventRecord(c->ev_phase[0], c->stream) != hipSuccess || hipEventRecord(c->ev_phase[1], c->stream) != hipSuccess) {
        delete c;
        return RSH_E_DEVICE;
    }
    if (ctx_warm(c) != hipSuccess || warm_calls(c) != RSH_OK) {
        (void)hipStreamSynchronize(c->stream);
        delete c;
        return RSH_E_DEVICE;
    }
    *out = c;
    return RSH_OK;
}

void rsh_ctx_destroy(rsh_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (hipStream_t st : {ctx->stream, ctx->aux, ctx->phase})  // nothing may still read or write its buffers
        if (st) (void)hipStreamSynchronize(st);
    delete ctx;
}

void* rsh_ctx_stream(rsh_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int rsh_ctx_sync(rsh_ctx* ctx) {
    if (!ctx) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->aux));    // includes a cancelled speculation draining
    RSH_HIP(hipStreamSynchronize(ctx->phase));  // a stopped phase-shifted speculation and its downloads
    return RSH_OK;
}

// The pass-sized buffers back to the device and host allocators (a Generator and a Sender context on one
// GPU each kept 2 x segment_bytes of HBM between segments).  Small round-trip buffers stay: they are what the next
// call would otherwise allocate on its latency path.
int rsh_ctx_trim(rsh_ctx* ctx) {
    if (!ctx) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    for (hipStream_t st : {ctx->stream, ctx->aux, ctx->phase}) RSH_HIP(hipStreamSynchronize(st));
    for (DevBuf* b : {&ctx->data, &ctx->weak, &ctx->strong, &ctx->seg_data, &ctx->seg_tab, &ctx->rcv[0], &ctx->rcv[1],
                      &ctx->rcv_ops[0], &ctx->rcv_ops[1], &ctx->out})
        b->release();
    for (PinnedBuf* b : {&ctx->h_stage, &ctx->h_rcv_ops[0], &ctx->h_rcv_ops[1], &ctx->h_out})
        b->release();
    if (ctx->h_win.cap > (1u << 20)) ctx->h_win.release();  // (a Receiver pass's pieces; the scan's windows are small)
    // The batched scan's state stays: its chunk index, hit map, descriptors, pinned event and
    // table buffers and fiber stacks are bounded by the largest segment's chunk count and option chain_map_bytes
    // (INTEGRATION.md "Per-context memory"), and rebuilding them cost the next segment scan ~3.4 ms of allocations.
    return RSH_OK;
}

// Generator.getBlockLengthFor / pow2SquareRoot (Generator.java:198-206, 219-236).
int32_t rsh_block_length_for(int64_t file_size) {
    if (file_size <= 0) return 0;
    const int exponent = 63 - __builtin_clzll((unsigned long long)file_size);
    const int32_t bl = (int32_t)(1u << (exponent / 2));
    return bl > 512 ? bl : 512;  // MIN_BLOCK_SIZE (:186)
}

// Generator.getDigestLength (:208-212) with Util.log2 = Math.log(n) / Math.log(2) (Util.java:128-130),
// then max(minDigestLength, ...) (:873).
int32_t rsh_digest_length_for(int64_t file_size, int32_t block_length, int32_t min_digest_length) {
    if (file_size <= 0) return 0;  // Generator.java:873: digestLength 0 for an empty file
    const int64_t lf = (int64_t)(__builtin_log((double)file_size) / __builtin_log(2.0));
    const int64_t lb = (int64_t)(__builtin_log((double)block_length) / __builtin_log(2.0));
    int32_t r = ((int32_t)(10 + 2 * lf - lb) - 24) / 8;
    r = std::min(r, 16);
    r = std::max(r, 2);
    return std::max(r, min_digest_length);
}

int rsh_header_make(int32_t block_length, int32_t digest_length, int64_t file_size, rsh_header* out) {
    if (!out || block_length < 0 || file_size < 0) return RSH_E_INVAL;
    if (block_length == 0) {
        *out = rsh_header{0, 0, 0, 0};
        return RSH_OK;
    }
    const int64_t rem = file_size % block_length;
    const int64_t cc = file_size / block_length + (rem > 0 ? 1 : 0);
    if (cc > 2147483647LL) return RSH_E_OVERFLOW;
    *out = rsh_header{(int32_t)cc, block_length, digest_length, (int32_t)rem};
    return RSH_OK;
}

// Checksum.Header 4-arg ctor (Checksum.java:75-92); IllegalArgumentException -> RsyncProtocolException
// in Connection.receiveChecksumHeader (Connection.java:28-38).
int rsh_header_validate(const rsh_header* h) {
    if (!h) return RSH_E_INVAL;
    if (h->chunk_count < 0) return RSH_E_PROTOCOL;
    if (h->block_length == 0 && h->chunk_count > 0) return RSH_E_PROTOCOL;
    if (h->block_length < 0 || h->block_length > kMaxBlockLength) return RSH_E_PROTOCOL;
    if (h->remainder < 0 || h->remainder > h->block_length) return RSH_E_PROTOCOL;
    if (h->digest_length < 0) return RSH_E_PROTOCOL;
    return RSH_OK;
}

int rsh_block_sums_device(rsh_ctx* ctx, const void* d_data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                          void* d_weak, void* d_strong) {
    if (!ctx || !seed) return RSH_E_INVAL;
    const int rc = check_generator_header(n, h);
    if (rc != RSH_OK) return rc;
    if (h->chunk_count == 0) return RSH_OK;
    if (!d_data || !d_weak || (!d_strong && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    // the K1's own start / stop timestamps (rsh_debug_kernel_ms; no marker packets around it; option time_gen)
    if (rsh::opt(rsh::OPT_TIME_GEN) != 0) rsh::k1_timing_next(ctx->ev_gen_a, ctx->ev_gen_b);
    const hipError_t e = rsh::launch_block_sums(static_cast<const uint8_t*>(d_data), n, (uint32_t)h->block_length,
                                                (uint32_t)h->chunk_count, (uint32_t)h->digest_length, seed_word(seed),
                                                static_cast<int32_t*>(d_weak), static_cast<uint8_t*>(d_strong),
                                                ctx->stream);
    ctx->gen_timed = rsh::k1_timing_taken();
    rsh::k1_timing_next(nullptr, nullptr);
    RSH_HIP(e);
    return RSH_OK;
}

int rsh_block_sums(rsh_ctx* ctx, const uint8_t* data, int64_t n, const rsh_header* h, const uint8_t seed[4],
                   int32_t* weak_out, uint8_t* strong_out) {
    if (!ctx || !seed) return RSH_E_INVAL;
    const int rc = check_generator_header(n, h);
    if (rc != RSH_OK) return rc;
    if (h->chunk_count == 0) return RSH_OK;
    if (!data || !weak_out || (!strong_out && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
    RSH_HIP(ctx->data.ensure((size_t)n));
    RSH_HIP(ctx->weak.ensure(C * 4));
    RSH_HIP(ctx->strong.ensure(C * dl + 1));
    RSH_HIP(hipMemcpyAsync(ctx->data.p, data, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    const int r2 = rsh_block_sums_device(ctx, ctx->data.p, n, h, seed, ctx->weak.p, ctx->strong.p);
    if (r2 != RSH_OK) return r2;
    RSH_HIP(hipMemcpyAsync(weak_out, ctx->weak.p, C * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (dl) RSH_HIP(hipMemcpyAsync(strong_out, ctx->strong.p, C * dl, hipMemcpyDeviceToHost, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_match_scan_device(rsh_ctx* ctx, const void* d_src, int64_t n, const rsh_header* h, const void* d_weak,
                          const void* d_strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap,
                          int64_t* n_ev, int64_t* literal, int64_t* matched, rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || n < 0) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    rsh::ResolveResult r;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        if (!d_src || (h->chunk_count > 0 && (!d_weak || (!d_strong && h->digest_length > 0)))) return RSH_E_INVAL;
        CallTrace tr("scan_call", n);  // with scan_device's teardown
        const int rc = scan_device(ctx, static_cast<const uint8_t*>(d_src), n, h, static_cast<const int32_t*>(d_weak),
                                   static_cast<const uint8_t*>(d_strong), nullptr, nullptr, seed, &r);
        if (rc != RSH_OK) return rc;
    }
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_match_scan(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                   const uint8_t* strong, const uint8_t seed[4], rsh_event* ev, int64_t ev_cap, int64_t* n_ev,
                   uint8_t file_md5[16], int64_t* literal, int64_t* matched, rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || !file_md5 || n < 0 || (n > 0 && !src)) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    // the whole-file digest (Sender.java:1241,1326) is one serial chain: host thread, beside the device
    std::thread md5_thread([&] {
        rsh::HostMd5 m;
        if (n > 0) m.update(src, (size_t)n);
        m.final(file_md5);
    });
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
        if (C > 0 && (!weak || (!strong && dl > 0))) rc = RSH_E_INVAL;
        if (rc == RSH_OK && (ctx->data.ensure((size_t)n) != hipSuccess || ctx->weak.ensure(C * 4 + 4) != hipSuccess ||
                             ctx->strong.ensure(C * dl + 1) != hipSuccess))
            rc = RSH_E_NOMEM;
        if (rc == RSH_OK) {
            bool okc = hipMemcpyAsync(ctx->data.p, src, (size_t)n, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C) okc = okc && hipMemcpyAsync(ctx->weak.p, weak, C * 4, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C && dl)
                okc = okc && hipMemcpyAsync(ctx->strong.p, strong, C * dl, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            rc = okc ? scan_device(ctx, ctx->data.as<uint8_t>(), n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(),
                                   weak, strong, seed, &r)
                     : RSH_E_DEVICE;
        }
    }
    md5_thread.join();
    if (rc != RSH_OK) return rc;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_match_scan_tiled(rsh_ctx* ctx, const uint8_t* src, int64_t n, const rsh_header* h, const int32_t* weak,
                         const uint8_t* strong, const uint8_t seed[4], int64_t tile_bytes, rsh_event* ev,
                         int64_t ev_cap, int64_t* n_ev, uint8_t file_md5[16], int64_t* literal, int64_t* matched,
                         rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || n < 0 || tile_bytes < 0 || (n > 0 && !src)) return RSH_E_INVAL;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    std::thread md5_thread;
    if (file_md5)
        md5_thread = std::thread([&] {
            rsh::HostMd5 m;
            if (n > 0) m.update(src, (size_t)n);
            m.final(file_md5);
        });
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (h->block_length == 0) {
        skip_events(n, &r);
    } else if (n > 0) {
        const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
        if (C > 0 && (!weak || (!strong && dl > 0))) rc = RSH_E_INVAL;
        if (rc == RSH_OK && (ctx->weak.ensure(C * 4 + 4) != hipSuccess || ctx->strong.ensure(C * dl + 1) != hipSuccess))
            rc = RSH_E_NOMEM;
        if (rc == RSH_OK) {
            bool okc = true;
            if (C) okc = hipMemcpyAsync(ctx->weak.p, weak, C * 4, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            if (C && dl)
                okc = okc && hipMemcpyAsync(ctx->strong.p, strong, C * dl, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
            auto fill = [&](uint8_t* dst, int64_t off, int64_t len) -> hipError_t {
                const hipError_t e = hipMemcpyAsync(dst, src + off, (size_t)len, hipMemcpyHostToDevice, ctx->stream);
                return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
            };
            const int64_t tb = tile_bytes > 0 ? tile_bytes : kDefaultTile;
            rc = okc ? scan_tiled(ctx, fill, n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(), weak, strong, seed,
                                  tb, &r)
                     : RSH_E_DEVICE;
        }
    }
    if (md5_thread.joinable()) md5_thread.join();
    if (rc != RSH_OK) return rc;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

int rsh_fetch_events(rsh_ctx* ctx, rsh_event* ev, int64_t ev_cap, int64_t* n_ev) {
    if (!ctx || !n_ev) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    *n_ev = (int64_t)ctx->last_ev.size();
    if (*n_ev > ev_cap || (!ev && *n_ev > 0)) return RSH_E_NOSPACE;
    if (*n_ev > 0) memcpy(ev, ctx->last_ev.data(), ctx->last_ev.size() * sizeof(rsh_event));
    return RSH_OK;
}

int rsh_file_md5(const uint8_t* data, int64_t n, uint8_t out[16]) {
    if (!out || n < 0 || (n > 0 && !data)) return RSH_E_INVAL;
    rsh::HostMd5 m;
    if (n > 0) m.update(data, (size_t)n);
    m.final(out);
    return RSH_OK;
}

int64_t rsh_tokens_size(const rsh_event* ev, int64_t n_ev) {
    int64_t size = 4 + 16;  // putInt(0) + file MD5
    for (int64_t i = 0; i < n_ev; ++i) {
        if (ev[i].kind == RSH_EV_LITERAL) size += ev[i].length + 4 * ((ev[i].length + kChunkSize - 1) / kChunkSize);
        else size += 4 * (int64_t)ev[i].count;
    }
    return size;
}

static inline uint8_t* put_int(uint8_t* o, int32_t v) {  // BufferedOutputChannel is little-endian (:50)
    for (int i = 0; i < 4; ++i) o[i] = (uint8_t)((uint32_t)v >> (8 * i));
    return o + 4;
}

int rsh_tokens_write(const uint8_t* src, const rsh_event* ev, int64_t n_ev, const uint8_t file_md5[16], uint8_t* out,
                     int64_t cap) {
    if (!out || !file_md5 || (n_ev > 0 && !ev)) return RSH_E_INVAL;
    if (rsh_tokens_size(ev, n_ev) > cap) return RSH_E_NOSPACE;
    uint8_t* o = out;
    for (int64_t i = 0; i < n_ev; ++i) {
        if (ev[i].kind == RSH_EV_LITERAL) {  // Sender.sendDataFrom (:794-809)
            if (!src) return RSH_E_INVAL;
            for (int64_t cur = ev[i].offset, end = ev[i].offset + ev[i].length; cur < end;) {
                const int64_t len = std::min<int64_t>(kChunkSize, end - cur);
                o = put_int(o, (int32_t)len);
                memcpy(o, src + cur, (size_t)len);
                o += len;
                cur += len;
            }
        } else {
            for (int32_t j = 0; j < ev[i].count; ++j) o = put_int(o, -(ev[i].index + j + 1));  // :1274
        }
    }
    o = put_int(o, 0);          // :1316
    memcpy(o, file_md5, 16);    // sendFiles :1148
    return RSH_OK;
}

int64_t rsh_generator_bytes(const rsh_header* h, const int32_t* weak, const uint8_t* strong, uint8_t* out, int64_t cap) {
    if (!h) return RSH_E_INVAL;
    const int64_t size = 16 + (int64_t)h->chunk_count * (4 + h->digest_length);
    if (!out) return size;
    if (cap < size || (h->chunk_count > 0 && (!weak || (!strong && h->digest_length > 0)))) return RSH_E_NOSPACE;
    uint8_t* o = out;
    o = put_int(o, h->chunk_count);  // Connection.sendChecksumHeader (Connection.java:40-45)
    o = put_int(o, h->block_length);
    o = put_int(o, h->digest_length);
    o = put_int(o, h->remainder);
    for (int32_t i = 0; i < h->chunk_count; ++i) {  // Generator.java:890-893
        o = put_int(o, weak[i]);
        memcpy(o, strong + (int64_t)i * h->digest_length, (size_t)h->digest_length);
        o += h->digest_length;
    }
    return size;
}

int rsh_dev_alloc(rsh_ctx* ctx, int64_t bytes, void** out) {
    if (!ctx || !out || bytes < 0) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    return hipMalloc(out, (size_t)(bytes ? bytes : 1)) == hipSuccess ? RSH_OK : RSH_E_NOMEM;
}

int rsh_dev_free(rsh_ctx* ctx, void* p) {
    if (!ctx) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    if (p) RSH_HIP(hipFree(p));
    return RSH_OK;
}

int rsh_memcpy_h2d(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (!ctx || bytes < 0 || (bytes > 0 && (!dst || !src))) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_memcpy_d2h(rsh_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (!ctx || bytes < 0 || (bytes > 0 && (!dst || !src))) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

int rsh_debug_set_option(const char* name, int64_t value) {
    const int i = rsh::opt_index(name);
    if (!rsh::opt_settable(i)) return RSH_E_INVAL;  // unknown, or an A/B switch outside the diagnostics build
    rsh::opt_table()[i].store(value, std::memory_order_relaxed);
    return RSH_OK;
}

int rsh_debug_get_option(const char* name, int64_t* value) {
    const int i = rsh::opt_index(name);
    if (i < 0 || !value) return RSH_E_INVAL;
    *value = rsh::opt((rsh::Opt)i);
    return RSH_OK;
}

void rsh_debug_reset_options(void) {
    for (int i = 0; i < rsh::OPT_COUNT; ++i) rsh::opt_table()[i].store(rsh::opt_info()[i].def, std::memory_order_relaxed);
}

int rsh_debug_kernel_ms(rsh_ctx* ctx, int32_t which, double* ms) {
    if (!ctx || !ms || which < 0 || which > 1) return RSH_E_INVAL;
    *ms = -1.0;
    const bool timed = which == 0 ? ctx->gen_timed : ctx->spec_timed;
    if (!timed) return RSH_OK;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(hipEventSynchronize(which == 0 ? ctx->ev_gen_b : ctx->ev_k1b));
    float f = 0.f;
    RSH_HIP(hipEventElapsedTime(&f, which == 0 ? ctx->ev_gen_a : ctx->ev_k1a, which == 0 ? ctx->ev_gen_b : ctx->ev_k1b));
    *ms = f;
    return RSH_OK;
}

int rsh_debug_generation(rsh_ctx* ctx, int32_t set, int32_t* gen) {
    if (!ctx || set < -1 || set > rsh_ctx::kGenWrapAt) return RSH_E_INVAL;
    if (set >= 0) ctx->gen = set;
    if (gen) *gen = ctx->gen;
    return RSH_OK;
}

int rsh_debug_streams_busy(rsh_ctx* ctx, int32_t* mask) {
    if (!ctx || !mask) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    *mask = 0;
    const hipStream_t st[3] = {ctx->stream, ctx->aux, ctx->phase};
    for (int i = 0; i < 3; ++i) {
        const hipError_t e = hipStreamQuery(st[i]);
        if (e == hipErrorNotReady) *mask |= 1 << i;
        else if (e != hipSuccess) RSH_HIP(e);
    }
    return RSH_OK;
}

int rsh_debug_k1_clock(rsh_ctx* ctx, const void* d_data, int64_t n, int32_t block_length, int32_t reps,
                       double* clock_ghz) {
    if (!ctx || !d_data || !clock_ghz || reps <= 0 || block_length <= 0 || n <= 0 || block_length % 128 != 0 ||
        n % (64 * (int64_t)block_length) != 0)
        return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    const int64_t C = n / block_length;
    void *w = nullptr, *st = nullptr, *clk = nullptr;
    hipError_t e = hipMalloc(&w, (size_t)C * 4);
    if (e == hipSuccess) e = hipMalloc(&st, (size_t)C * 16);
    if (e == hipSuccess) e = hipMalloc(&clk, 16);
    if (e == hipSuccess) e = hipMemsetAsync(clk, 0, 16, ctx->stream);
    for (int32_t r = 0; e == hipSuccess && r < reps; ++r)
        e = rsh::launch_k1_clock(static_cast<const uint8_t*>(d_data), n, (uint32_t)block_length, 16, 0x04030201u,
                                 static_cast<int32_t*>(w), static_cast<uint8_t*>(st),
                                 static_cast<unsigned long long*>(clk), ctx->stream);
    unsigned long long h[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(h, clk, 16, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    for (void* p : {w, st, clk})
        if (p) (void)hipFree(p);
    RSH_HIP(e);
    *clock_ghz = h[1] ? 0.1 * (double)h[0] / (double)h[1] : 0.0;  // ticks / (ticks of 10 ns) / 10 ns -> GHz
    return RSH_OK;
}

int rsh_fill_splitmix_device(rsh_ctx* ctx, void* d_out, int64_t n, uint64_t key, int64_t byte_offset) {
    if (!ctx || (n > 0 && !d_out) || n < 0 || byte_offset < 0) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    RSH_HIP(rsh::launch_fill_splitmix(static_cast<uint8_t*>(d_out), n, key, byte_offset, ctx->stream));
    return RSH_OK;
}

}  // extern "C"
