// pieces.cpp -- the two passes over a file handed over as a list of host buffers ("pieces") instead of one
// contiguous array.  A JVM cannot hold a BASELINE-size file in one direct ByteBuffer (capacity is an int:
// at most 2^31 - 1 bytes), while the reference streams any file size through FileView's 10*B window
// (FileView.java:51-80,235-278; Sender.java:1105-1110).  The binding therefore reads the file into pieces of
// at most 1 GiB and the library treats their concatenation as the file:
//   * the Generator (Generator.java:886-895) assembles the basis in HBM a tile at a time -- a chunk may
//     straddle two pieces, never a tile (tiles are multiples of B);
//   * the Sender (Sender.java:1235-1327) assembles the source in HBM (or pages it a tile at a time above
//     file_tile_above, as rsh_match_scan_tiled does) while a host thread digests the pieces in order (the
//     whole-file MD5, Sender.java:1241,1326).
// Events and sums are those of rsh_block_sums / rsh_match_scan on the concatenated bytes.
#include <thread>

#include "ctx.h"
#include "host_md5.h"
#include "options.h"

namespace {

// Sources up to file_tile_above (32 GiB) are assembled whole in HBM, larger ones a tile of file_tile (4 GiB) at a
// time; the Generator always goes tile by tile (options.h, the thresholds rsh_match_scan_file uses: tests lower
// them to run the tiled paths at small sizes).
int64_t resident_max() { return rsh::opt(rsh::OPT_FILE_TILE_ABOVE); }
int64_t tile_bytes() { return std::max<int64_t>(16, rsh::opt(rsh::OPT_FILE_TILE)); }

// Validates the piece list and returns the total byte count (or a negative status).
int64_t pieces_total(const rsh_piece* pieces, int32_t npieces) {
    if (npieces < 0 || (npieces > 0 && !pieces)) return RSH_E_INVAL;
    int64_t n = 0;
    for (int32_t i = 0; i < npieces; ++i) {
        if (pieces[i].len < 0 || (pieces[i].len > 0 && !pieces[i].data)) return RSH_E_INVAL;
        n += pieces[i].len;
    }
    return n;
}

// Copies bytes [off, off + len) of the concatenated pieces to device memory dst (enqueued on s).
hipError_t copy_range(const rsh_piece* pieces, int32_t npieces, int64_t off, int64_t len, uint8_t* dst, hipStream_t s) {
    int64_t base = 0;
    for (int32_t i = 0; i < npieces && len > 0; ++i) {
        const int64_t pl = pieces[i].len;
        if (off < base + pl) {
            const int64_t a = off - base, take = std::min(len, pl - a);
            const hipError_t e = hipMemcpyAsync(dst, pieces[i].data + a, (size_t)take, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return e;
            dst += take;
            off += take;
            len -= take;
        }
        base += pl;
    }
    return hipSuccess;
}

void pieces_md5(const rsh_piece* pieces, int32_t npieces, uint8_t out[16]) {
    rsh::HostMd5 m;
    for (int32_t i = 0; i < npieces; ++i)
        if (pieces[i].len > 0) m.update(pieces[i].data, (size_t)pieces[i].len);
    m.final(out);
}

}  // namespace

namespace rsh {

// The Generator pass over pieces, the context claimed by the caller (rsh_block_sums_pieces; segment.cpp for a
// segment's file too large for one pass).  n = the pieces' total.
int block_sums_pieces_claimed(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, int64_t n, const rsh_header* h,
                              const uint8_t seed[4], int32_t* weak_out, uint8_t* strong_out) {
    if (h->chunk_count == 0) return RSH_OK;
    if (!weak_out || (!strong_out && h->digest_length > 0)) return RSH_E_INVAL;
    RSH_HIP(hipSetDevice(ctx->device));
    const int64_t B = h->block_length, C = h->chunk_count, dl = h->digest_length;
    // two tiles in HBM: the next one is copied while the previous one is summed
    const int64_t T = std::max<int64_t>(B, std::min<int64_t>(n, tile_bytes()) / B * B);
    const int64_t ntiles = (n + T - 1) / T;
    RSH_HIP(ctx->data.ensure((size_t)(ntiles > 1 ? 2 * T : n)));
    RSH_HIP(ctx->weak.ensure((size_t)C * 4));
    RSH_HIP(ctx->strong.ensure((size_t)(C * dl + 1)));
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t lo = t * T, len = std::min(T, n - lo), c0 = lo / B;
        uint8_t* db = ctx->data.as<uint8_t>() + (t & 1) * T;
        // the tile's buffer was last read by the launch two tiles back, which precedes this copy on the stream
        RSH_HIP(copy_range(pieces, npieces, lo, len, db, ctx->stream));
        RSH_HIP(rsh::launch_block_sums(db, len, (uint32_t)B, (uint32_t)((len + B - 1) / B), (uint32_t)dl,
                                       seed_word(seed), ctx->weak.as<int32_t>() + c0,
                                       ctx->strong.as<uint8_t>() + c0 * dl, ctx->stream));
    }
    RSH_HIP(hipMemcpyAsync(weak_out, ctx->weak.p, (size_t)C * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (dl > 0) RSH_HIP(hipMemcpyAsync(strong_out, ctx->strong.p, (size_t)(C * dl), hipMemcpyDeviceToHost, ctx->stream));
    RSH_HIP(hipStreamSynchronize(ctx->stream));
    return RSH_OK;
}

// The Sender scan over pieces without the whole-file digest, the context claimed by the caller; h validated,
// block_length > 0, n > 0.  The source is assembled in HBM, or paged through it a tile at a time above
// file_tile_above.
int scan_pieces_claimed(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, int64_t n, const rsh_header* h,
                        const int32_t* weak, const uint8_t* strong, const uint8_t seed[4], ResolveResult* r) {
    const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
    const bool resident = n <= resident_max();
    if (ctx->weak.ensure(C * 4 + 4) != hipSuccess || ctx->strong.ensure(C * dl + 1) != hipSuccess ||
        (resident && ctx->data.ensure((size_t)n) != hipSuccess))
        return RSH_E_NOMEM;
    hipError_t e = hipSuccess;
    int rc = RSH_OK;
    if (C) e = hipMemcpyAsync(ctx->weak.p, weak, C * 4, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && C && dl) e = hipMemcpyAsync(ctx->strong.p, strong, C * dl, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && resident) {
        e = copy_range(pieces, npieces, 0, n, ctx->data.as<uint8_t>(), ctx->stream);
        if (e == hipSuccess)
            rc = scan_device(ctx, ctx->data.as<uint8_t>(), n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(),
                             weak, strong, seed, r);
    } else if (e == hipSuccess) {  // larger than we keep in HBM whole: one tile at a time
        auto fill = [&](uint8_t* dst, int64_t off, int64_t len) -> hipError_t {
            const hipError_t e2 = copy_range(pieces, npieces, off, len, dst, ctx->stream);
            return e2 != hipSuccess ? e2 : hipStreamSynchronize(ctx->stream);
        };
        rc = scan_tiled(ctx, fill, n, h, ctx->weak.as<int32_t>(), ctx->strong.as<uint8_t>(), weak, strong, seed,
                        tile_bytes(), r);
    }
    if (e != hipSuccess) {
        note_error(e, __LINE__, "pieces.cpp");
        return RSH_E_DEVICE;
    }
    return rc;
}

}  // namespace rsh

extern "C" {

int rsh_block_sums_pieces(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, const rsh_header* h,
                          const uint8_t seed[4], int32_t* weak_out, uint8_t* strong_out) {
    if (!ctx || !seed) return RSH_E_INVAL;
    const int64_t n = pieces_total(pieces, npieces);
    if (n < 0) return (int)n;
    const int rc = check_generator_header(n, h);
    if (rc != RSH_OK) return rc;
    if (h->chunk_count == 0) return RSH_OK;
    RSH_CLAIM(ctx);
    return rsh::block_sums_pieces_claimed(ctx, pieces, npieces, n, h, seed, weak_out, strong_out);
}

int rsh_match_scan_pieces(rsh_ctx* ctx, const rsh_piece* pieces, int32_t npieces, const rsh_header* h,
                          const int32_t* weak, const uint8_t* strong, const uint8_t seed[4], rsh_event* ev,
                          int64_t ev_cap, int64_t* n_ev, uint8_t file_md5[16], int64_t* literal, int64_t* matched,
                          rsh_scan_stats* stats) {
    if (!ctx || !h || !seed || !n_ev || !file_md5) return RSH_E_INVAL;
    const int64_t n = pieces_total(pieces, npieces);
    if (n < 0) return (int)n;
    const int v = rsh_header_validate(h);
    if (v != RSH_OK) return v;
    const size_t C = (size_t)h->chunk_count, dl = (size_t)h->digest_length;
    if (h->block_length > 0 && n > 0 && C > 0 && (!weak || (!strong && dl > 0))) return RSH_E_INVAL;
    RSH_CLAIM(ctx);
    RSH_HIP(hipSetDevice(ctx->device));
    std::thread md5_thread([&] { pieces_md5(pieces, npieces, file_md5); });  // one serial chain, beside the scan
    rsh::ResolveResult r;
    int rc = RSH_OK;
    if (h->block_length == 0) skip_events(n, &r);
    else if (n > 0) rc = rsh::scan_pieces_claimed(ctx, pieces, npieces, n, h, weak, strong, seed, &r);
    md5_thread.join();
    if (rc != RSH_OK) return rc;
    if (literal) *literal = r.literal;
    if (matched) *matched = r.matched;
    if (stats) *stats = r.stats;
    return emit_events(ctx, r, ev, ev_cap, n_ev);
}

}  // extern "C"
